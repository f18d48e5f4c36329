"""A8 local bundle adjustment: HIP kernels (k_ba.hip) vs the oracle (oracle/numpy_ba.py).

Same rendered sequence through the HIP engine and through ``OracleTracker`` + ``BATracker``.
Bar: keyframe slots, landmark ids and observations (u, v, disparity) identical (integer / copied
values); observation and landmark counts of the last solve identical; keyframe poses and landmark
positions within 1e-9 relative of the oracle (measured: 2e-15 and 3e-14) (the solves
use Cholesky and fixed-order sums where the oracle uses LU and numpy's order; the stated
product tolerance is 1e-4).
"""

from __future__ import annotations

import functools

import numpy as np
import pytest

from helpers import rel_frobenius, scenario

pytestmark = pytest.mark.gpu

BA_ITEMS = (("ba_window", 4), ("ba_kf_interval", 2), ("ba_iters", 3), ("ba_lambda", 1.0), ("ba_outlier_px", 3.0))


@functools.lru_cache(maxsize=2)
def _scenario_and_oracle(n: int):
    sc = scenario(seed=0, n=n, cfg_items=BA_ITEMS)
    return sc, _oracle_windows(sc)


def _imu_factors(sc, n: int, angle: float = 3e-3, weight: float = 1e5) -> dict:
    """Per keyframe g > 0: the front end's rotation from keyframe g - interval to g, turned by
    `angle` about z (so the factor pulls), and its weight."""
    iv = sc["cfg"].ba_kf_interval
    Rz = np.array([[np.cos(angle), -np.sin(angle), 0.0], [np.sin(angle), np.cos(angle), 0.0], [0.0, 0.0, 1.0]])
    out = {}
    for g in range(iv, n, iv):
        Rc = np.linalg.inv(sc["oracle"][g]["world_T_cam"])[:3, :3]
        Rp = np.linalg.inv(sc["oracle"][g - iv]["world_T_cam"])[:3, :3]
        out[g] = (Rz @ Rc @ Rp.T, weight)
    return out


# gravity, accelerometer-bias prior and weight, gyroscope-bias prior and weight (oldest keyframe)
INE_CFG = (np.array([0.4, 9.7, 1.2]), np.array([0.01, 0.0, -0.01]), 10.0, np.array([0.0, 0.002, 0.0]), 100.0)
B_TRUE = np.array([0.02, -0.01, 0.03, 0.004, -0.003, 0.002])   # accelerometer, gyroscope biases


def _inertial_factors(sc, n: int) -> dict:
    """Per keyframe g > 0: an inertial factor whose velocity, position and gyro-rotation residuals
    vanish at the oracle front end's cameras, central-difference velocities and the biases B_TRUE
    (the BA's visual window disagrees slightly, so the factors pull), with the initial velocity
    off by 0.05 m/s."""
    from helpers import exact_inertial_record

    rng = np.random.default_rng(7)
    iv = sc["cfg"].ba_kf_interval
    dt = iv / 30.0
    gw = INE_CFG[0]
    Tcw = [np.linalg.inv(r["world_T_cam"]) for r in sc["oracle"]]
    pos = [r["world_T_cam"][:3, 3] for r in sc["oracle"]]
    vel = {g: (pos[min(g + 1, n - 1)] - pos[max(g - 1, 0)]) / (dt / iv * (min(g + 1, n - 1) - max(g - 1, 0)))
           for g in range(0, n, iv)}
    out = {}
    for g in range(iv, n, iv):
        f = exact_inertial_record(Tcw[g - iv], vel[g - iv], Tcw[g], vel[g], gw, dt, B_TRUE, rng)
        out[g] = (f, vel[g] + rng.normal(0, 0.05, 3))
    return out


def _oracle_windows(sc, imu: dict | None = None, ine: dict | None = None):
    from oracle.numpy_ba import BAParams, BATracker

    cfg, rect = sc["cfg"], sc["rect"]
    bp = BAParams(window=cfg.ba_window, kf_interval=cfg.ba_kf_interval, iters=cfg.ba_iters, lam=cfg.ba_lambda,
                  outlier_px=cfg.ba_outlier_px)
    trk = BATracker(cfg.n_features, (rect.fx, rect.fy, rect.cx, rect.cy, rect.fx * rect.baseline), bp)
    if ine is not None:
        trk.win.set_inertial(*INE_CFG)
    snaps = []
    for g, res in enumerate(sc["oracle"]):
        trk.step(res, imu=None if imu is None else imu.get(g), ine=None if ine is None else ine.get(g))
        w = trk.win
        snaps.append({"frames": w.frame.copy(), "T_cw": w.T_cw.copy(), "lm": w.lm.copy(), "X": w.X.copy(),
                      "u": w.u.copy(), "v": w.v.copy(), "d": w.d.copy(), "solve": trk.last_solve,
                      "vel": w.vel.copy(), "bias": w.bias.copy()})
    return snaps


def _compare(got: dict, want: dict, where: str):
    np.testing.assert_array_equal(got["frames"], want["frames"], err_msg=where)
    occ = want["frames"] >= 0
    np.testing.assert_array_equal(got["lm"][occ], want["lm"][occ], err_msg=where)
    for key in ("u", "v", "d"):
        np.testing.assert_array_equal(got[key][occ], want[key][occ], err_msg=f"{where} {key}")
    for s in np.nonzero(occ)[0]:
        assert rel_frobenius(got["T_cw"][s], want["T_cw"][s]) < 1e-9, (where, s)
    ids = np.unique(want["lm"][occ])
    ids = ids[ids >= 0]
    assert ids.size > 0
    err = np.linalg.norm(got["X"][ids] - want["X"][ids], axis=1) / np.linalg.norm(want["X"][ids], axis=1)
    assert err.max() < 1e-9, (where, float(err.max()))
    if want["solve"] is not None and want["solve"]["n_obs"]:
        assert got["n_obs"] == want["solve"]["n_obs"] and got["n_lm"] == want["solve"]["n_lm"], where
        assert got["ok"]


@pytest.mark.parametrize("batch", [12, 3])
def test_ba_window_parity(batch):
    import torch

    from thor_slam_amd._lib import Handle

    n = 12   # 6 keyframes through a 4-slot window: two evictions
    sc, want = _scenario_and_oracle(n)
    h = Handle([sc["rect"]], sc["cfg"], max_batch=batch)
    dev = torch.from_numpy(np.ascontiguousarray(sc["frames"])).cuda()
    try:
        for b0 in range(0, n, batch):
            nb = min(batch, n - b0)
            h.submit(dev[b0:].data_ptr(), nb, torch.cuda.current_stream().cuda_stream)
            _compare(h.ba_read(0), want[b0 + nb - 1], f"after frame {b0 + nb - 1}")
    finally:
        h.close()
    assert (want[-1]["frames"] >= 0).all()
    assert want[-1]["solve"]["n_lm"] > 50


def test_ba_split_solve_equals_fused_handoff():
    """The in-launch hand-off of k_ba_reduce_solve (write-through stores + agent-scope loads, no
    kernel boundary) against the same reduction and solve split across a kernel
    boundary (tslam_ba_split_solve): windows, poses and landmarks bit-identical, and the IMU
    factor path (it reads the window poses in the solve block) too."""
    import torch

    from thor_slam_amd._lib import Handle

    n, batch = 12, 3
    sc, _ = _scenario_and_oracle(n)
    imu = _imu_factors(sc, n)
    dev = torch.from_numpy(np.ascontiguousarray(sc["frames"])).cuda()
    runs = {}
    for split in (False, True):
        h = Handle([sc["rect"]], sc["cfg"], max_batch=batch)
        try:
            h.ba_split_solve(split)
            for g, (M, w) in imu.items():
                h.ba_imu_factor(g, M, w)
            snaps = []
            for b0 in range(0, n, batch):
                h.submit(dev[b0:].data_ptr(), batch, torch.cuda.current_stream().cuda_stream)
                snaps.append(h.ba_read(0))
            runs[split] = (snaps, h.read_poses(batch))
        finally:
            h.close()
    for k, (a, b) in enumerate(zip(runs[False][0], runs[True][0])):
        for key in ("frames", "lm", "T_cw", "X"):
            np.testing.assert_array_equal(np.asarray(a[key]).view(np.uint8), np.asarray(b[key]).view(np.uint8),
                                          err_msg=f"batch {k} {key}")
        assert a["ok"] and b["ok"] and a["n_lm"] == b["n_lm"] > 50
    for key, a in runs[False][1].items():   # the last batch's published poses
        np.testing.assert_array_equal(a, runs[True][1][key], err_msg=key)


@pytest.mark.parametrize("split", [False, True])
def test_ba_graph_replay_equals_direct_launches(split):
    """tslam_ba_graph: each keyframe's chain replayed from a captured hipGraph
    whose kernels read the keyframe's record (the default) against the direct by-value launches:
    30 keyframes through the 4-slot window in batches of 6 with IMU rotation and inertial factors
    on — more replays of the steady-state chain than an instance ring holds (24), so instances are
    re-pointed at new records — windows, velocities, bias and poses bit-identical."""
    import torch

    from thor_slam_amd._lib import Handle

    n, batch = 60, 6
    sc = scenario(seed=0, n=n, cfg_items=BA_ITEMS)
    imu, ine = _imu_factors(sc, n), _inertial_factors(sc, n)
    dev = torch.from_numpy(np.ascontiguousarray(sc["frames"])).cuda()
    runs = {}
    for graph in (False, True):
        h = Handle([sc["rect"]], sc["cfg"], max_batch=batch)
        try:
            h.ba_graph(graph)
            h.ba_split_solve(split)
            h.ba_inertial(*INE_CFG)
            for g, (M, w) in imu.items():
                h.ba_imu_factor(g, M, w)
            for g, (f, v0) in ine.items():
                h.ba_inertial_factor(g, f, v0)
            snaps = []
            for b0 in range(0, n, batch):
                h.submit(dev[b0:].data_ptr(), batch, torch.cuda.current_stream().cuda_stream)
                snaps.append((h.ba_read(0), h.ba_read_inertial(0)))
            runs[graph] = (snaps, h.read_poses(batch))
        finally:
            h.close()
    for k, ((a, ai), (b, bi)) in enumerate(zip(runs[False][0], runs[True][0])):
        for key in ("frames", "lm", "T_cw", "X"):
            np.testing.assert_array_equal(np.asarray(a[key]).view(np.uint8), np.asarray(b[key]).view(np.uint8),
                                          err_msg=f"batch {k} {key}")
        np.testing.assert_array_equal(ai["vel"], bi["vel"])
        np.testing.assert_array_equal(ai["bias"], bi["bias"])
        assert a["ok"] and a["n_lm"] == b["n_lm"] > 50
    for key, a in runs[False][1].items():
        np.testing.assert_array_equal(a, runs[True][1][key], err_msg=key)


def test_ba_imu_rotation_factors_parity():
    """IMU rotation factors between window-consecutive keyframes (tslam_ba_imu_factor) against the
    oracle's imu_terms: same windows to 1e-9, through evictions, in batches of 3 — and the factors
    move the solution (it differs from the vision-only window)."""
    import torch

    from thor_slam_amd._lib import Handle

    n, batch = 12, 3
    sc, plain = _scenario_and_oracle(n)
    imu = _imu_factors(sc, n)
    want = _oracle_windows(sc, imu)
    h = Handle([sc["rect"]], sc["cfg"], max_batch=batch)
    dev = torch.from_numpy(np.ascontiguousarray(sc["frames"])).cuda()
    try:
        for g, (M, w) in imu.items():
            h.ba_imu_factor(g, M, w)
        for b0 in range(0, n, batch):
            h.submit(dev[b0:].data_ptr(), batch, torch.cuda.current_stream().cuda_stream)
            _compare(h.ba_read(0), want[b0 + batch - 1], f"imu factors, after frame {b0 + batch - 1}")
    finally:
        h.close()
    occ = want[-1]["frames"] >= 0
    moved = max(rel_frobenius(want[-1]["T_cw"][s_], plain[-1]["T_cw"][s_]) for s_ in np.nonzero(occ)[0])
    assert moved > 1e-6, moved


def test_ba_inertial_factors_parity():
    """Tightly coupled inertial factors (tslam_ba_inertial / _inertial_factor: velocities per
    keyframe and the window's accelerometer bias eliminated into the camera system,
    k_ba_reduce_solve_ine) against the oracle's inertial_terms: windows, velocities and bias to
    1e-9 through evictions, in batches of 3, with the IMU rotation factors on too; the factors
    move the solution; the split (kernel-boundary) solve agrees bit for bit."""
    import torch

    from thor_slam_amd._lib import Handle

    n, batch = 12, 3
    sc, plain = _scenario_and_oracle(n)
    imu = _imu_factors(sc, n)
    ine = _inertial_factors(sc, n)
    want = _oracle_windows(sc, imu, ine)
    dev = torch.from_numpy(np.ascontiguousarray(sc["frames"])).cuda()
    runs = []
    for split in (False, True):
        h = Handle([sc["rect"]], sc["cfg"], max_batch=batch)
        try:
            h.ba_split_solve(split)
            h.ba_inertial(*INE_CFG)
            for g, (M, w) in imu.items():
                h.ba_imu_factor(g, M, w)
            for g, (f, v0) in ine.items():
                h.ba_inertial_factor(g, f, v0)
            snaps = []
            for b0 in range(0, n, batch):
                h.submit(dev[b0:].data_ptr(), batch, torch.cuda.current_stream().cuda_stream)
                got = h.ba_read(0)
                want_k = want[b0 + batch - 1]
                _compare(got, want_k, f"inertial, after frame {b0 + batch - 1}")
                gi = h.ba_read_inertial(0)
                occ = want_k["frames"] >= 0
                err_v = np.abs(gi["vel"][occ] - want_k["vel"][occ]).max() / np.abs(want_k["vel"][occ]).max()
                assert err_v < 1e-9, (b0, err_v)
                err_b = np.abs(gi["bias"][occ] - want_k["bias"][occ]).max()
                assert err_b < 1e-9 * max(np.abs(want_k["bias"][occ]).max(), 1e-3), (b0, err_b)
                snaps.append((got, gi))
            runs.append(snaps)
        finally:
            h.close()
    for (a, ai), (b, bi) in zip(*runs):
        np.testing.assert_array_equal(a["T_cw"], b["T_cw"])
        np.testing.assert_array_equal(ai["vel"], bi["vel"])
        np.testing.assert_array_equal(ai["bias"], bi["bias"])
    occ = want[-1]["frames"] >= 0
    moved = max(rel_frobenius(want[-1]["T_cw"][s_], plain[-1]["T_cw"][s_]) for s_ in np.nonzero(occ)[0])
    assert moved > 1e-7, moved
    occ = want[-1]["frames"] >= 0
    assert np.abs(want[-1]["bias"][occ][:, 3:6]).max() > 1e-4   # the gyroscope biases moved off zero


def test_ba_two_pairs_own_factors_parity():
    """Two independent stereo pairs (no rig) fed the same frames, each window with its own
    keyframe factors — pair 0 IMU rotation + inertial factors, pair 1 other rotation factors only —
    each against its own oracle window to 1e-9 through evictions.  The keyframe insertion runs in
    each pair's solve launch (k_ba_insert_gate), so this pins that every pair's factors reach its
    own window and nothing leaks from one pair into the other."""
    import torch

    from thor_slam_amd._lib import Handle

    n, batch = 12, 3
    sc, _ = _scenario_and_oracle(n)
    imu0, imu1 = _imu_factors(sc, n), _imu_factors(sc, n, angle=-2e-3, weight=5e4)
    ine = _inertial_factors(sc, n)
    want = (_oracle_windows(sc, imu0, ine), _oracle_windows(sc, imu1))
    frames = np.ascontiguousarray(np.concatenate([sc["frames"], sc["frames"]], axis=1))   # [n][4][H][W]
    dev = torch.from_numpy(frames).cuda()
    h = Handle([sc["rect"], sc["rect"]], sc["cfg"], max_batch=batch)
    try:
        h.ba_inertial(*INE_CFG, pair=0)
        for g, (M, w) in imu0.items():
            h.ba_imu_factor(g, M, w, pair=0)
        for g, (M, w) in imu1.items():
            h.ba_imu_factor(g, M, w, pair=1)
        for g, (f, v0) in ine.items():
            h.ba_inertial_factor(g, f, v0, pair=0)
        for b0 in range(0, n, batch):
            h.submit(dev[b0:].data_ptr(), batch, torch.cuda.current_stream().cuda_stream)
            for p in (0, 1):
                _compare(h.ba_read(p), want[p][b0 + batch - 1], f"pair {p}, after frame {b0 + batch - 1}")
            gi, wk = h.ba_read_inertial(0), want[0][b0 + batch - 1]
            occ = wk["frames"] >= 0
            assert np.abs(gi["vel"][occ] - wk["vel"][occ]).max() < 1e-9 * np.abs(wk["vel"][occ]).max()
    finally:
        h.close()
    a0, a1 = want[0][-1], want[1][-1]
    occ = a0["frames"] >= 0
    assert max(rel_frobenius(a0["T_cw"][s_], a1["T_cw"][s_]) for s_ in np.nonzero(occ)[0]) > 1e-7   # the windows differ


def test_ba_deferred_issue_equals_immediate():
    """tslam_ba_defer: the stage API pipelined as bench.py --config c4 drives it (front stages on
    one stream, back stages on a second, the BA stage on a third) with each batch's BA launches
    enqueued at the next batch's first back stage instead of inside the BA stage call.  Windows,
    landmarks and the last batch's poses are bit-identical to the immediate issue, and equal the
    oracle's windows."""
    import torch

    from thor_slam_amd._lib import Handle

    n, batch = 12, 3
    sc, want = _scenario_and_oracle(n)
    dev = torch.from_numpy(np.ascontiguousarray(sc["frames"])).cuda()
    front, back, bas = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()
    runs = {}
    for defer in (False, True):
        h = Handle([sc["rect"]], sc["cfg"], max_batch=batch)
        try:
            h.ba_defer(defer)
            for b0 in range(0, n, batch):
                h.begin_batch(dev[b0:].data_ptr(), batch)
                for st, stream in (("rectify", front), ("detect", front), ("describe", front), ("match", back), ("pose", back)):
                    h.run_stage(st, stream.cuda_stream)
                h.run_stage("ba", bas.cuda_stream)
                h.end_batch()
            got = h.ba_read(0)   # flushes a deferred BA, then synchronises
            runs[defer] = (got, h.read_poses(batch))
        finally:
            h.close()
    for key in ("frames", "lm", "T_cw", "X"):
        np.testing.assert_array_equal(np.asarray(runs[False][0][key]).view(np.uint8),
                                      np.asarray(runs[True][0][key]).view(np.uint8), err_msg=key)
    for key, a in runs[False][1].items():
        np.testing.assert_array_equal(a, runs[True][1][key], err_msg=key)
    _compare(runs[True][0], want[n - 1], "deferred, last batch")


def test_ba_inertial_state_resets_and_rejects_bad_input():
    """tslam_reset clears the window's velocities and accelerometer bias (a new session), and
    tslam_ba_inertial_factor refuses a non-finite record, dt <= 0 or a negative weight."""
    import torch

    from thor_slam_amd._lib import Handle

    n, batch = 12, 3
    sc, _ = _scenario_and_oracle(n)
    ine = _inertial_factors(sc, n)
    h = Handle([sc["rect"]], sc["cfg"], max_batch=batch)
    dev = torch.from_numpy(np.ascontiguousarray(sc["frames"])).cuda()
    try:
        f, v0 = ine[2]
        for bad in (np.where(np.arange(f.size) == 3, np.nan, f), np.where(np.arange(f.size) == 27, 0.0, f),
                    np.where(np.arange(f.size) == 29, -1.0, f), np.where(np.arange(f.size) == 71, -1.0, f),
                    np.where(np.arange(f.size) == 45, np.inf, f)):
            with pytest.raises(RuntimeError, match="tslam error"):
                h.ba_inertial_factor(2, bad, v0)
        with pytest.raises(RuntimeError, match="tslam error"):
            h.ba_inertial_factor(2, f, np.array([np.inf, 0.0, 0.0]))
        h.ba_inertial(*INE_CFG)
        for g, (rec, v) in ine.items():
            h.ba_inertial_factor(g, rec, v)
        for b0 in range(0, n, batch):
            h.submit(dev[b0:].data_ptr(), batch, torch.cuda.current_stream().cuda_stream)
        got = h.ba_read_inertial(0)
        assert np.abs(got["bias"]).max() > 0 and np.abs(got["vel"]).max() > 0
        h.reset()
        got = h.ba_read_inertial(0)
        np.testing.assert_array_equal(got["vel"], 0.0)
        np.testing.assert_array_equal(got["bias"], 0.0)
    finally:
        h.close()


def test_ba_imu_factor_rejects_non_finite():
    """tslam_ba_imu_factor refuses an infinite / NaN weight or rotation entry (they would poison the
    window's whole Schur system) and leaves the window unchanged."""
    from thor_slam_amd._lib import Handle

    sc, _ = _scenario_and_oracle(12)
    h = Handle([sc["rect"]], sc["cfg"], max_batch=2)
    try:
        M = np.eye(3)
        for Mx, w in ((M, np.inf), (M, np.nan), (M, -1.0), (np.full((3, 3), np.nan), 1.0), (M * np.inf, 1.0)):
            with pytest.raises(RuntimeError, match="tslam error"):
                h.ba_imu_factor(5, Mx, w)
        h.ba_imu_factor(5, M, 1e3)   # finite: accepted
    finally:
        h.close()


def test_ba_stage_is_idempotent_per_batch():
    """Running the BA stage again for the same batch inserts nothing twice."""
    import torch

    from thor_slam_amd._lib import Handle

    sc, want = _scenario_and_oracle(12)
    h = Handle([sc["rect"]], sc["cfg"], max_batch=4)
    dev = torch.from_numpy(np.ascontiguousarray(sc["frames"])).cuda()
    stream = torch.cuda.current_stream().cuda_stream
    try:
        h.begin_batch(dev.data_ptr(), 4)
        h.run_stage("all", stream)
        h.run_stage("ba", stream)
        h.end_batch()
        got = h.ba_read(0)
        np.testing.assert_array_equal(got["frames"], [0, 2, -1, -1])
        _compare(got, want[3], "frames 0-3, BA stage twice")
    finally:
        h.close()


def test_engine_publishes_ba_poses_and_map():
    """HipSlamEngine with local BA: each published pose is the front end carried by its newest
    window keyframe's correction (the oracle's window at that frame), get_map returns every
    keyframe and the window's landmarks, and the drift against ground truth shrinks."""
    from thor_slam_amd.camera import CameraRig, Extrinsics
    from thor_slam_amd.params import HipSlamConfig
    from thor_slam_amd.slam.hip_engine import HipSlamEngine

    from helpers import make_source

    n = 12
    sc, want = _scenario_and_oracle(n)
    src = make_source(0)
    rig = CameraRig([src], rig_extrinsics={src.name: Extrinsics.from_4x4_matrix(src.rig_T_source)})
    rig.start()
    eng = HipSlamEngine(num_cameras=2, config=HipSlamConfig(batch_size=1, **dict(BA_ITEMS)))
    eng.initialize(rig.calibration)
    bt = src.rig_T_source @ src.get_extrinsics()[0].to_4x4_matrix() @ sc["rect"].left_optical_T_rect()
    inv = np.linalg.inv
    poses = []
    for g in range(n):
        pose = eng.process_frames(rig.get_synchronized_frames())
        poses.append(pose)
        w = want[g]
        live = {int(f): inv(w["T_cw"][s]) for s, f in enumerate(w["frames"]) if f >= 0}
        kf = max(f for f in live if f <= g)
        fe = sc["oracle"]
        expect = bt @ live[kf] @ inv(fe[kf]["world_T_cam"]) @ fe[g]["world_T_cam"] @ inv(bt)
        assert rel_frobenius(pose.to_4x4_matrix(), expect) < 1e-9, g
    smap = eng.get_map()
    assert [round(p.timestamp, 6) for p in smap.keyframe_poses] == sorted(round(p.timestamp, 6) for p in smap.keyframe_poses)
    assert len(smap.keyframe_poses) == n // 2
    assert len(smap.points) == np.unique(want[-1]["lm"][want[-1]["lm"] >= 0]).size
    assert all(p.observations >= 1 for p in smap.points)
    gt = inv(src.ground_truth_body(0)) @ src.ground_truth_body(n - 1)
    fe_err = np.linalg.norm((bt @ sc["oracle"][n - 1]["world_T_cam"] @ inv(bt))[:3, 3] - gt[:3, 3])
    assert np.linalg.norm(poses[-1].position - gt[:3, 3]) < fe_err
    eng.shutdown()


@pytest.mark.parametrize("mapping,cap", [(True, 50), (False, 100000)])
def test_engine_map_size_and_mapping_switch(mapping, cap):
    """SlamConfig.max_map_size bounds the persistent map, enable_mapping=False keeps none
    (reference fields thor_slam/slam/interface.py:110-111); poses are unaffected."""
    from thor_slam_amd.camera import CameraRig, Extrinsics
    from thor_slam_amd.params import HipSlamConfig
    from thor_slam_amd.slam.hip_engine import HipSlamEngine

    from helpers import make_source

    src = make_source(0)
    rig = CameraRig([src], rig_extrinsics={src.name: Extrinsics.from_4x4_matrix(src.rig_T_source)})
    rig.start()
    eng = HipSlamEngine(num_cameras=2, config=HipSlamConfig(batch_size=1, enable_mapping=mapping, max_map_size=cap,
                                                            **dict(BA_ITEMS)))
    eng.initialize(rig.calibration)
    for _ in range(8):
        eng.process_frames(rig.get_synchronized_frames())
    smap = eng.get_map()
    assert len(smap.points) == (cap if mapping else 0)
    assert len(smap.keyframe_poses) == 4
    eng.shutdown()


def test_ba_on_its_own_stream_matches():
    """The BA stage on a second stream, overlapping the next batches' front end (the library
    orders it with events and a pose snapshot): same windows as the oracle."""
    import torch

    from thor_slam_amd._lib import Handle

    n, batch = 12, 3
    sc, want = _scenario_and_oracle(n)
    h = Handle([sc["rect"]], sc["cfg"], max_batch=batch)
    dev = torch.from_numpy(np.ascontiguousarray(sc["frames"])).cuda()
    main, side = torch.cuda.current_stream(), torch.cuda.Stream()
    try:
        for b0 in range(0, n, batch):
            h.begin_batch(dev[b0:].data_ptr(), batch)
            for st in ("rectify", "detect", "describe", "match", "pose"):
                h.run_stage(st, main.cuda_stream)
            h.run_stage("ba", side.cuda_stream)
            h.end_batch()
        _compare(h.ba_read(0), want[n - 1], "two streams, final window")
    finally:
        h.close()


C4_ITEMS = (("n_features", 4000), ("ba_window", 10), ("ba_kf_interval", 5), ("ba_iters", 5), ("ba_lambda", 1.0),
            ("ba_outlier_px", 3.0))


@pytest.mark.slow
def test_ba_window_parity_c4():
    """BASELINE.json configs[3] (C4) as bench.py --config c4 runs it: 1280x800, K=4000, a
    10-keyframe window with a keyframe every 5 frames and 5 Gauss-Newton iterations, batches of
    50 frames; 56 frames = 12 keyframes, so the full 10-slot window is solved and then evicts
    twice.  Compared with the oracle after every batch (frames 49 and 55)."""
    import torch

    from thor_slam_amd._lib import Handle

    n, batch = 56, 50
    sc = scenario(seed=0, n=n, width=1280, height=800, cfg_items=C4_ITEMS)
    want = _oracle_windows(sc)
    h = Handle([sc["rect"]], sc["cfg"], max_batch=batch)
    dev = torch.from_numpy(np.ascontiguousarray(sc["frames"])).cuda()
    try:
        for b0 in range(0, n, batch):
            nb = min(batch, n - b0)
            h.submit(dev[b0:].data_ptr(), nb, torch.cuda.current_stream().cuda_stream)
            _compare(h.ba_read(0), want[b0 + nb - 1], f"after frame {b0 + nb - 1}")
    finally:
        h.close()
    assert (want[-1]["frames"] >= 0).all() and want[-1]["frames"].min() == 10   # keyframes 0 and 5 evicted
    assert want[-1]["solve"]["n_lm"] > 1000
