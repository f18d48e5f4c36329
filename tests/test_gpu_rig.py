"""Rig pose: generalised PnP over every pair of a multi-source rig,
HIP ``k_rig_pose`` vs ``oracle/numpy_rig.py`` on the two-source bracket rig.

Bar: status, the winning candidate and the inlier count identical (the candidates start from
per-pair poses that agree with the oracle to ~1e-16; a borderline inlier could flip in principle,
none does on these frames), body motions and chained world_T_base within 1e-9 relative Frobenius.
"""

from __future__ import annotations

import functools

import numpy as np
import pytest

from helpers import C3_SOURCES, rel_frobenius, rig_scene
from oracle import numpy_slam as O
from oracle.numpy_rig import RigChain, rig_pose
from thor_slam_amd.params import HipSlamConfig

pytestmark = pytest.mark.gpu
NAMES = ("192.168.2.21", "192.168.2.25")


@functools.lru_cache(maxsize=2)
def rig_scenario(n: int = 6, names: tuple = NAMES):
    sc = dict(rig_scene(tuple(names), n))
    frames, rects, E = sc["frames"], sc["rects"], sc["E"]
    cfg = HipSlamConfig()
    trks = [O.OracleTracker(cfg, dict(fx=r.fx, fy=r.fy, cx=r.cx, cy=r.cy, baseline=r.baseline, map_l=r.map_left,
                                      map_r=r.map_right)) for r in rects]
    chain = RigChain()
    want = []
    for i in range(n):
        outs = [trk.step(frames[i, 2 * q], frames[i, 2 * q + 1]) for q, trk in enumerate(trks)]
        if i == 0:
            want.append({"status": 2, "T_abs": np.eye(4)})
            continue
        items = [{"status": o["status"], "T": o["T"], "corr": o.get("corr"),
                  "intr": (r.fx, r.fy, r.cx, r.cy)} for o, r in zip(outs, rects)]
        res = rig_pose(items, E, cfg)
        res["T_abs"] = chain.step(res)
        want.append(res)
    return {"frames": frames, "rects": rects, "E": E, "cfg": cfg, "want": want, "traj": sc["traj"]}


@pytest.mark.parametrize("batch", [6, 2])
def test_rig_pose_matches_oracle(batch):
    import torch

    from thor_slam_amd._lib import Handle

    sc = rig_scenario()
    h = Handle(sc["rects"], sc["cfg"], max_batch=batch)
    h.set_rig(sc["E"])
    dev = torch.from_numpy(np.ascontiguousarray(sc["frames"])).cuda()
    n = dev.shape[0]
    got = []
    for b0 in range(0, n, batch):
        nb = min(batch, n - b0)
        h.submit(dev[b0:].data_ptr(), nb, torch.cuda.current_stream().cuda_stream)
        r = h.read_rig_poses(nb)
        got += [{k: r[k][f] for k in r} for f in range(nb)]
    h.close()
    for i, (g, w) in enumerate(zip(got, sc["want"])):
        assert g["stats"][0] == w["status"], i
        if i == 0:
            continue
        assert g["stats"][4] == w["best"] and int(g["stats"][2]) == w["n_inliers"], (i, g["stats"], w)
        assert rel_frobenius(g["T_rel"], w["T"]) < 1e-9, i
        assert rel_frobenius(g["T_abs"], w["T_abs"]) < 1e-9, i
        assert rel_frobenius(g["cov"], w["cov"]) < 1e-6, i
    # and the joint solve tracks the rendered body motion
    gt = np.linalg.inv(sc["traj"][0]) @ sc["traj"][n - 1]
    assert np.linalg.norm(got[-1]["T_abs"][:3, 3] - gt[:3, 3]) < 0.1 * np.linalg.norm(gt[:3, 3]) + 2e-3


def test_rig_pose_survives_a_blind_pair():
    """One pair sees a blank wall (no correspondences): the rig still tracks from the other."""
    import torch

    from thor_slam_amd._lib import Handle

    sc = rig_scenario()
    frames = sc["frames"].copy()
    frames[:, 2:] = 128   # pair 1 blind
    h = Handle(sc["rects"], sc["cfg"], max_batch=6)
    h.set_rig(sc["E"])
    dev = torch.from_numpy(np.ascontiguousarray(frames)).cuda()
    h.submit(dev.data_ptr(), 6, torch.cuda.current_stream().cuda_stream)
    r = h.read_rig_poses(6)
    per = h.read_poses(6)
    h.close()
    assert (per["stats"][1:, 1, 0] != 0).all()          # the blind pair is lost
    assert (r["stats"][1:, 0] == 0).all()               # the rig is not
    gt = np.linalg.inv(sc["traj"][0]) @ sc["traj"][5]
    assert np.linalg.norm(r["T_abs"][5][:3, 3] - gt[:3, 3]) < 0.1 * np.linalg.norm(gt[:3, 3]) + 2e-3


def check_rig_against_oracle(sc, got):
    for i, (g, w) in enumerate(zip(got, sc["want"])):
        assert g["stats"][0] == w["status"], i
        if i == 0:
            continue
        assert g["stats"][4] == w["best"] and int(g["stats"][2]) == w["n_inliers"], (i, g["stats"], w)
        assert rel_frobenius(g["T_rel"], w["T"]) < 1e-9, i
        assert rel_frobenius(g["T_abs"], w["T_abs"]) < 1e-9, i
        assert rel_frobenius(g["cov"], w["cov"]) < 1e-6, i


def test_c3_eight_stream_rig_matches_oracle():
    """BASELINE.json configs[2] (C3): the four OAK sources of run_slam.py:45-50 on the
    brackets.urdf joints, 8 streams / 4 stereo pairs, one handle on one GPU, 5 frames against the
    oracle's per-pair trackers + rig pose (oracle/numpy_rig.py)."""
    import torch

    from thor_slam_amd._lib import Handle

    sc = rig_scenario(5, C3_SOURCES)
    assert sc["frames"].shape[1] == 8
    h = Handle(sc["rects"], sc["cfg"], max_batch=5)
    h.set_rig(sc["E"])
    dev = torch.from_numpy(np.ascontiguousarray(sc["frames"])).cuda()
    h.submit(dev.data_ptr(), 5, torch.cuda.current_stream().cuda_stream)
    r = h.read_rig_poses(5)
    h.close()
    check_rig_against_oracle(sc, [{k: r[k][f] for k in r} for f in range(5)])
    assert (r["stats"][1:, 0] == 0).all()
