"""Rig-level A8: one window of body poses over the keyframes of every
pair of the two-source bracket rig, HIP (k_ba.hip rig kernels) vs ``oracle/numpy_ba.py``
(``RigKeyframeWindow`` / ``RigBATracker``), driven by the oracle's per-pair tracking and rig chain.

Bar: keyframe slots, landmark ids and observations identical (integer / copied values); every
pair's cameras and the body poses within 1e-9 relative Frobenius, landmark positions within 1e-9
relative (the stated product tolerance is 1e-4); each pair's cameras stay at E_p^-1 B.
"""

from __future__ import annotations

import functools

import numpy as np
import pytest

from helpers import rel_frobenius, rig_scene
from oracle import numpy_slam as O
from oracle.numpy_ba import BAParams, RigBATracker
from oracle.numpy_rig import RigChain, inv_rigid, rig_pose
from thor_slam_amd.params import HipSlamConfig

pytestmark = pytest.mark.gpu
NAMES = ("192.168.2.21", "192.168.2.25")
BA_ITEMS = dict(ba_window=4, ba_kf_interval=2, ba_iters=3, ba_lambda=1.0, ba_outlier_px=3.0)
N = 10


# gravity, accelerometer-bias prior and weight, gyroscope-bias prior and weight (oldest keyframe)
RIG_INE_CFG = (np.array([0.3, -9.75, 0.9]), np.array([0.0, 0.01, 0.0]), 10.0, np.array([0.001, 0.0, 0.0]), 100.0)


def _body_inertial_factors(T_abs: list) -> dict:
    """Per body keyframe g > 0: an inertial factor (body axes) whose velocity, position and
    gyro-rotation residuals vanish at the rig chain's body poses, central-difference velocities and
    biases (0.02, -0.01, 0.03 | 0.003, 0.002, -0.004); initial velocities off by 0.05 m/s (the BA's
    visual window disagrees slightly: the factors pull)."""
    from helpers import exact_inertial_record

    rng = np.random.default_rng(11)
    iv = BA_ITEMS["ba_kf_interval"]
    dt = 1.0 / 30.0
    gw = RIG_INE_CFG[0]
    b_true = np.array([0.02, -0.01, 0.03, 0.003, 0.002, -0.004])
    Tbw = [inv_rigid(t) for t in T_abs]
    pos = [t[:3, 3] for t in T_abs]
    vel = {g: (pos[min(g + 1, N - 1)] - pos[max(g - 1, 0)]) / (dt * (min(g + 1, N - 1) - max(g - 1, 0)))
           for g in range(0, N, iv)}
    out = {}
    for g in range(iv, N, iv):
        f = exact_inertial_record(Tbw[g - iv], vel[g - iv], Tbw[g], vel[g], gw, iv * dt, b_true, rng)
        out[g] = (f, vel[g] + rng.normal(0, 0.05, 3))
    return out


@functools.lru_cache(maxsize=2)
def rig_ba_scenario(inertial: bool = False):
    ine = _body_inertial_factors(rig_ba_scenario()["T_abs"]) if inertial else None
    sc = dict(rig_scene(NAMES, N))
    frames, rects, E = sc["frames"], sc["rects"], sc["E"]
    cfg = HipSlamConfig(**BA_ITEMS)
    trks = [O.OracleTracker(cfg, dict(fx=r.fx, fy=r.fy, cx=r.cx, cy=r.cy, baseline=r.baseline, map_l=r.map_left,
                                      map_r=r.map_right)) for r in rects]
    bp = BAParams(window=cfg.ba_window, kf_interval=cfg.ba_kf_interval, iters=cfg.ba_iters, lam=cfg.ba_lambda,
                  outlier_px=cfg.ba_outlier_px)
    intrs = [(r.fx, r.fy, r.cx, r.cy, r.fx * r.baseline) for r in rects]
    ba = RigBATracker(cfg.n_features, intrs, E, bp)
    if ine is not None:
        ba.win.set_inertial(*RIG_INE_CFG)
    chain = RigChain()
    snaps, T_seq = [], []
    for i in range(N):
        outs = [trk.step(frames[i, 2 * q], frames[i, 2 * q + 1]) for q, trk in enumerate(trks)]
        if i == 0:
            T_abs = np.eye(4)
        else:
            items = [{"status": o["status"], "T": o["T"], "corr": o.get("corr"), "intr": (r.fx, r.fy, r.cx, r.cy)}
                     for o, r in zip(outs, rects)]
            T_abs = chain.step(rig_pose(items, E, cfg))
        T_seq.append(T_abs.copy())
        ba.step(i, outs, T_abs, ine=None if ine is None else ine.get(i))
        w = ba.win
        snaps.append({"frames": w.frame.copy(), "B": w.B.copy(), "solve": ba.last_solve,
                      "vel": w.vel.copy(), "bias": w.bias.copy(),
                      "pairs": [{"T_cw": pw.T_cw.copy(), "lm": pw.lm.copy(), "X": pw.X.copy(), "u": pw.u.copy(),
                                 "v": pw.v.copy(), "d": pw.d.copy()} for pw in w.pairs]})
    return {"frames": frames, "rects": rects, "E": E, "cfg": cfg, "snaps": snaps, "traj": sc["traj"], "T_abs": T_seq,
            "ine": ine}


def _compare(h, want: dict, E, where: str):
    P = len(E)
    body = h.ba_read(P)
    np.testing.assert_array_equal(body["frames"], want["frames"], err_msg=where)
    occ = want["frames"] >= 0
    for s in np.nonzero(occ)[0]:
        assert rel_frobenius(body["T_cw"][s], want["B"][s]) < 1e-9, (where, "body", s)
    for p in range(P):
        got, wp = h.ba_read(p), want["pairs"][p]
        np.testing.assert_array_equal(got["lm"][occ], wp["lm"][occ], err_msg=f"{where} pair {p}")
        for key in ("u", "v", "d"):
            np.testing.assert_array_equal(got[key][occ], wp[key][occ], err_msg=f"{where} pair {p} {key}")
        for s in np.nonzero(occ)[0]:
            assert rel_frobenius(got["T_cw"][s], wp["T_cw"][s]) < 1e-9, (where, p, s)
            assert rel_frobenius(got["T_cw"][s], inv_rigid(E[p]) @ body["T_cw"][s]) < 1e-12, (where, p, s)
        ids = np.unique(wp["lm"][occ])
        ids = ids[ids >= 0]
        assert ids.size > 0, (where, p)
        err = np.linalg.norm(got["X"][ids] - wp["X"][ids], axis=1) / np.linalg.norm(wp["X"][ids], axis=1)
        assert err.max() < 1e-9, (where, p, float(err.max()))
    if want["solve"] is not None and want["solve"]["n_obs"]:
        assert body["n_obs"] == want["solve"]["n_obs"] and body["n_lm"] == want["solve"]["n_lm"], where
        assert body["ok"], where


@pytest.mark.parametrize("batch", [N, 3])
def test_rig_ba_matches_oracle(batch):
    import torch

    from thor_slam_amd._lib import Handle

    sc = rig_ba_scenario()
    h = Handle(sc["rects"], sc["cfg"], max_batch=batch)
    h.set_rig(sc["E"])
    dev = torch.from_numpy(np.ascontiguousarray(sc["frames"])).cuda()
    for b0 in range(0, N, batch):
        nb = min(batch, N - b0)
        h.submit(dev[b0:].data_ptr(), nb, torch.cuda.current_stream().cuda_stream)
        h.read_poses(nb)
        _compare(h, sc["snaps"][b0 + nb - 1], sc["E"], f"after frame {b0 + nb - 1}")
    h.close()


def test_rig_ba_body_inertial_factors_match_oracle():
    """Inertial factors on the rig's body window (tslam_ba_inertial_factor with pair = n_pairs):
    body poses, every pair's cameras and landmarks, body velocities and the window's bias within
    1e-9 of RigKeyframeWindow's inertial solve, in batches of 3; pair windows are refused."""
    import torch

    from thor_slam_amd._lib import Handle

    sc = rig_ba_scenario(True)
    plain = rig_ba_scenario()
    P, batch = len(sc["E"]), 3
    h = Handle(sc["rects"], sc["cfg"], max_batch=batch)
    try:
        h.set_rig(sc["E"])
        with pytest.raises(RuntimeError, match="body window"):
            h.ba_inertial(*RIG_INE_CFG, pair=0)
        h.ba_inertial(*RIG_INE_CFG, pair=P)
        for g, (f, v0) in sc["ine"].items():
            h.ba_inertial_factor(g, f, v0, pair=P)
        dev = torch.from_numpy(np.ascontiguousarray(sc["frames"])).cuda()
        for b0 in range(0, N, batch):
            nb = min(batch, N - b0)
            h.submit(dev[b0:].data_ptr(), nb, torch.cuda.current_stream().cuda_stream)
            want = sc["snaps"][b0 + nb - 1]
            _compare(h, want, sc["E"], f"inertial, after frame {b0 + nb - 1}")
            gi = h.ba_read_inertial(P)
            occ = want["frames"] >= 0
            err_v = np.abs(gi["vel"][occ] - want["vel"][occ]).max() / max(np.abs(want["vel"][occ]).max(), 1e-3)
            assert err_v < 1e-9, (b0, err_v)
            err_b = np.abs(gi["bias"][occ] - want["bias"][occ]).max()
            assert err_b < 1e-9 * max(np.abs(want["bias"][occ]).max(), 1e-3), (b0, err_b)
    finally:
        h.close()
    last, base = sc["snaps"][-1], plain["snaps"][-1]
    occ = last["frames"] >= 0
    assert max(rel_frobenius(last["B"][s], base["B"][s]) for s in np.nonzero(occ)[0]) > 1e-7
    assert np.abs(last["bias"][last["frames"] >= 0]).max() > 1e-4


def test_rig_ba_every_pair_contributes():
    """Both pairs' landmarks enter the joint solve, and the window holds the evicted-then-refilled
    slots (5 keyframes through a 4-slot window)."""
    sc = rig_ba_scenario()
    last = sc["snaps"][-1]
    assert (last["frames"] >= 0).sum() == 4 and 0 not in last["frames"]
    per = last["solve"]["pairs"]
    assert len(per) == 2 and all(r["n_obs"] > 0 and r["n_lm"] > 0 for r in per)


def test_engine_publishes_the_rig_body_window():
    """HipSlamEngine on the two-source rig with local BA: the window is the body window, get_map
    returns the body keyframes (in-window ones = the device's BA estimates) and every pair's
    landmarks, and a keyframe frame's published pose is its BA body pose."""
    import json
    from pathlib import Path

    import torch

    from thor_slam_amd.camera import CameraRig, Extrinsics
    from thor_slam_amd.slam.hip_engine import HipSlamEngine

    sc = rig_scene(NAMES, N)
    mats = json.loads((Path(__file__).parent / "golden" / "brackets_joints.json").read_text())
    srcs = sc["sources"]
    rig = CameraRig(srcs, rig_extrinsics={s.name: Extrinsics.from_4x4_matrix(np.array(mats[s.name])) for s in srcs})
    cfg = HipSlamConfig(batch_size=N, **BA_ITEMS)
    eng = HipSlamEngine(num_cameras=4, config=cfg)
    eng.initialize(rig.calibration, cfg)
    assert len(eng._pairs) == 2
    dev = torch.from_numpy(np.ascontiguousarray(sc["frames"])).cuda()
    stamps = [srcs[0].timestamp(i) for i in range(N)]
    eng.process_batch(dev[: N - 1], stamps[: N - 1])   # ends on keyframe 8
    latest = eng._latest_pose.to_4x4_matrix()
    body = eng._handle.ba_read(2)
    s8 = int(np.nonzero(body["frames"] == 8)[0][0])
    assert rel_frobenius(latest, np.linalg.inv(body["T_cw"][s8])) < 1e-9
    eng.process_batch(dev[N - 1:], stamps[N - 1:])
    smap = eng.get_map()
    # frames 2, 4, 6, 8: keyframe 0 was inserted and evicted inside the first batch, before the
    # engine read the window (as for one pair)
    assert len(smap.keyframe_poses) == 4
    body = eng._handle.ba_read(2)
    by_stamp = {p.timestamp: p.to_4x4_matrix() for p in smap.keyframe_poses}
    for s_, f in enumerate(body["frames"]):
        if f >= 0:
            assert rel_frobenius(by_stamp[stamps[f]], np.linalg.inv(body["T_cw"][s_])) < 1e-12
    n_pts = 0
    for p in range(2):
        w = eng._handle.ba_read(p)
        occ = w["frames"] >= 0
        ids = np.unique(w["lm"][occ])
        n_pts += int((ids >= 0).sum())
    assert len(smap.points) == n_pts and n_pts > 0
    # and the published trajectory follows the rendered body motion (world = base at frame 0)
    gt = np.linalg.inv(sc["traj"][0]) @ sc["traj"][N - 1]
    got = eng._latest_pose.to_4x4_matrix()
    assert np.linalg.norm(got[:3, 3] - gt[:3, 3]) < 0.1 * np.linalg.norm(gt[:3, 3]) + 2e-3
    eng.shutdown()
