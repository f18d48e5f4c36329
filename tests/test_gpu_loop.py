"""Loop closure + keyframe pose graph on the device against
``oracle/numpy_loop.py``:

* the keyframe database (compacted stereo landmarks) is bit-exact, place-recognition votes are
  identical, verification gives the same RANSAC winner / counts and cam_q_T_cam_c within 1e-9;
* the device pose graph (dense normal equations, blocked Cholesky with FP64-MFMA trailing
  updates) equals the oracle's Gauss-Newton within 1e-9 relative, from 1 node to 200 nodes;
* HipSlamEngine closes the loop of a circular trajectory and the pose graph pulls the keyframes
  towards the rendered ground truth; on the two-source bracket rig place recognition runs over
  every pair's keyframe entries, so a loop only pair 1 can see is still closed."""

from __future__ import annotations

from concurrent.futures import ProcessPoolExecutor

import numpy as np
import pytest

from helpers import rel_frobenius
from oracle import numpy_loop as L
from oracle import numpy_slam as O
from thor_slam_amd.calib import extract_cameras, stereo_pairs, stereo_rectify
from thor_slam_amd.camera import CameraRig, Extrinsics
from thor_slam_amd.params import HipSlamConfig
from thor_slam_amd.synthetic import SyntheticStereoSource, circle_trajectory

pytestmark = pytest.mark.gpu

LOOP_FRAMES = 270          # 45 deg/s: the body is back at its start pose at frame 240
YAW = 45.0


def _loop_source():
    return SyntheticStereoSource(seed=0, trajectory=circle_trajectory(LOOP_FRAMES, yaw_rate_deg=YAW))


def _render(idx):
    src = _loop_source()
    return [src.render_stereo_sequence(1, start=i)[0] for i in idx]


def _render_many(frames_idx, workers=16):
    chunks = [frames_idx[i::workers] for i in range(workers) if frames_idx[i::workers]]
    out = {}
    with ProcessPoolExecutor(max_workers=len(chunks)) as ex:
        for c, frs in zip(chunks, ex.map(_render, chunks)):
            out.update(zip(c, frs))
    return np.stack([out[i] for i in frames_idx])


def _rect(src):
    cams = extract_cameras(CameraRig([src]).calibration, 2)
    (li, ri), = stereo_pairs(cams)
    return stereo_rectify(cams[li], cams[ri])


def _random_graph(rng, N, loops, noise=0.002):
    gt = [np.eye(4)]
    for _ in range(1, N):
        gt.append(gt[-1] @ L.se3_exp(np.r_[rng.normal(0, 0.1, 3), rng.normal(0, 0.05, 3)]))
    edges = [(i, i + 1) for i in range(N - 1)] + list(loops)
    Z = np.array([L.inv_se3(gt[i]) @ gt[j] @ L.se3_exp(rng.normal(0, noise, 6)) for i, j in edges])
    T0 = [np.eye(4)]
    for k in range(N - 1):
        T0.append(T0[-1] @ Z[k])
    info = np.array([L.loop_information(0.01, 0.005) * rng.uniform(0.5, 2.0) for _ in edges])
    return np.array(T0), np.array(edges), Z, info


@pytest.mark.parametrize("N,loops", [(1, []), (2, []), (30, [(0, 29), (4, 21)]),
                                     (200, [(0, 199), (10, 150), (50, 120), (3, 90), (60, 61)])])
def test_pose_graph_matches_oracle(N, loops):
    from thor_slam_amd._lib import Handle

    rng = np.random.default_rng(N)
    T0, edges, Z, info = _random_graph(rng, N, loops)
    src = _loop_source()
    h = Handle([_rect(src)], HipSlamConfig(), max_batch=1)
    got = h.pose_graph(T0, edges.reshape(-1, 2), Z.reshape(-1, 4, 4), info.reshape(-1, 6, 6), 6)
    h.close()
    want = L.optimize(T0, edges.reshape(-1, 2), Z.reshape(-1, 4, 4), info.reshape(-1, 6, 6), 6)
    np.testing.assert_array_equal(got["T"][0], T0[0])   # the gauge node never moves
    for i in range(N):
        assert rel_frobenius(got["T"][i], want["T"][i]) < 1e-9, i
    if len(edges):
        assert abs(got["cost"] - want["cost"]) <= 1e-9 * max(want["cost"], 1e-12) + 1e-18
        assert want["steps"][-1] < 1e-8   # converged, so the comparison is at the optimum


def test_pose_graph_rejects_bad_graphs():
    from thor_slam_amd._lib import Handle

    h = Handle([_rect(_loop_source())], HipSlamConfig(), max_batch=1)
    T = np.array([np.eye(4)] * 3)
    with pytest.raises(RuntimeError, match="no edge"):
        h.pose_graph(T, np.array([[0, 1]]), np.array([np.eye(4)]), np.array([np.eye(6)]), 2)
    with pytest.raises(RuntimeError, match="bad edge"):
        h.pose_graph(T, np.array([[0, 3]]), np.array([np.eye(4)]), np.array([np.eye(6)]), 2)
    h.close()


def test_degenerate_span_is_singular_on_the_device():
    """A span with a free gauge direction (test_oracle_loop_policy.degenerate_span: zero residuals,
    the last edge informs translation only) fails the device's Cholesky exactly where the oracle's
    does: TSLAM_ESINGULAR (SingularSystemError) from the synchronous solve and from a loop job,
    after which the handle solves a well-posed graph as before."""
    from test_oracle_loop_policy import degenerate_span
    from thor_slam_amd._lib import Handle, SingularSystemError

    T, edges, Z, info = degenerate_span()
    with pytest.raises(np.linalg.LinAlgError):
        L.optimize(T, edges, Z, info, 3)
    h = Handle([_rect(_loop_source())], HipSlamConfig(), max_batch=1)
    with pytest.raises(SingularSystemError, match="not positive definite"):
        h.pose_graph(T, edges, Z, info, 3)
    h.loop_init(64, 256)
    job = h.loop_job_pose_graph(T, edges, Z, info, 3)
    with pytest.raises(SingularSystemError):
        job.result(block=True)
    T0, e0, Z0, i0 = _random_graph(np.random.default_rng(30), 30, [(0, 29), (4, 21)])
    got = h.pose_graph(T0, e0, Z0, i0, 6)
    want = L.optimize(T0, e0, Z0, i0, 6)
    assert max(rel_frobenius(a, b) for a, b in zip(got["T"], want["T"])) < 1e-9
    h.close()


def test_potrf_late_blocks_read_the_unfactored_tile():
    """Regression for the k_pg_potrf diagonal-tile race (fixed in round 5): with
    tslam_test_potrf_delay every block >= 1 of each panel launch reads A_kk only after block 0
    has stored its factor (~100 us late), the read order under which the former in-place store of
    L_kk handed late blocks a factored tile.  The solve must be bit-identical to the undelayed
    one and equal the oracle's Gauss-Newton (a 200-node graph: 38 tile panels)."""
    from thor_slam_amd._lib import Handle, load_library

    lib = load_library()
    rng = np.random.default_rng(200)
    T0, edges, Z, info = _random_graph(rng, 200, [(0, 199), (10, 150), (50, 120), (3, 90)])
    h = Handle([_rect(_loop_source())], HipSlamConfig(), max_batch=1)
    base = h.pose_graph(T0, edges, Z, info, 4)
    assert lib.tslam_test_potrf_delay(30) == 0
    try:
        late = h.pose_graph(T0, edges, Z, info, 4)
    finally:
        assert lib.tslam_test_potrf_delay(0) == 0
    h.close()
    np.testing.assert_array_equal(late["T"], base["T"])
    assert late["cost"] == base["cost"]
    want = L.optimize(T0, edges, Z, info, 4)
    assert max(rel_frobenius(a, b) for a, b in zip(late["T"], want["T"])) < 1e-9


def test_keyframe_database_votes_and_verification():
    import torch

    from thor_slam_amd._lib import Handle

    src = _loop_source()
    rect = _rect(src)
    cfg = HipSlamConfig()
    picks = [0, 60, 120, 180, 240, 245]
    frames = np.stack([src.render_stereo_sequence(1, start=g)[0] for g in picks])
    h = Handle([rect], cfg, max_batch=len(picks))
    h.loop_init(16, 256)
    dev = torch.from_numpy(frames).cuda()
    h.submit(dev.data_ptr(), len(picks), torch.cuda.current_stream().cuda_stream)
    intr = (rect.fx, rect.fy, rect.cx, rect.cy, rect.fx * rect.baseline)
    ora = []
    for k in range(len(picks)):
        trk = O.OracleTracker(cfg, dict(fx=rect.fx, fy=rect.fy, cx=rect.cx, cy=rect.cy, baseline=rect.baseline,
                                        map_l=rect.map_left, map_r=rect.map_right))
        cur = trk.step(frames[k, 0], frames[k, 1])["cur"]
        ora.append((cur, L.keyframe_landmarks(cur["left"], cur["disp"], intr)))
        slot, n = h.loop_add_keyframe(k)
        assert slot == k and n == ora[k][1]["xyz"].shape[0] > 1000
        got = h.loop_read_keyframe(slot)
        np.testing.assert_array_equal(got["desc"], ora[k][1]["desc"])
        np.testing.assert_array_equal(got["xyz"], ora[k][1]["xyz"])   # same IEEE operations: bit-exact
    for q in (4, 5):   # frames 240 / 245 revisit frame 0's place
        votes = h.loop_query(q, 4)
        want = [L.vote(ora[q][1]["desc"], ora[j][1]["desc"], 256, cfg.max_hamming, cfg.ratio_pct) for j in range(4)]
        np.testing.assert_array_equal(votes, want)
        assert L.best_candidate(votes, 4, cfg.loop_min_votes) == 0
        ver = h.loop_verify(q, 0)
        o = L.verify(ora[q][0]["left"], ora[0][1], intr[:4], cfg, q)
        assert ver["stats"][0] == o["status"] == 0
        assert ver["stats"][1] == o["n_corr"] and ver["stats"][2] == o["n_inliers"] and ver["stats"][4] == o["best_hyp"]
        assert rel_frobenius(ver["T"], o["T"]) < 1e-9
        # against the rendered ground truth: cam_q_T_cam_0 (rect frames = camera frames here)
        bt = src.rig_T_source @ src.get_extrinsics()[0].to_4x4_matrix() @ rect.left_optical_T_rect()
        gt = np.linalg.inv(bt) @ np.linalg.inv(src.ground_truth_body(picks[q])) @ src.ground_truth_body(0) @ bt
        assert np.linalg.norm(ver["T"][:3, 3] - gt[:3, 3]) < 0.02
    h.close()


@pytest.mark.slow
def test_engine_closes_the_loop():
    import torch

    from thor_slam_amd.slam.hip_engine import HipSlamEngine

    src = _loop_source()
    frames = _render_many(list(range(LOOP_FRAMES)))
    cfg = HipSlamConfig(batch_size=30, enable_loop_closure=True)
    eng = HipSlamEngine(num_cameras=2, config=cfg)
    rig = CameraRig([src], rig_extrinsics={src.name: Extrinsics.from_4x4_matrix(src.rig_T_source)})
    eng.initialize(rig.calibration, cfg)   # base_link = the FLU body of the ground truth
    dev = torch.from_numpy(frames).cuda()
    for b0 in range(0, LOOP_FRAMES, 30):
        eng.process_batch(dev[b0:b0 + 30], [src.timestamp(i) for i in range(b0, b0 + 30)])
    eng.settle()   # the searches of the last keyframes (due loop_latency frames later)
    loops = eng.loop_closures
    assert loops, "no loop closed"
    assert all(c <= 40 and q >= 225 for c, q, _ in loops), loops
    pg = eng.pose_graph
    lp = eng._loop
    bt = eng._base_T_rect
    gt0 = np.linalg.inv(src.ground_truth_body(0))
    err_raw, err_opt = [], []
    for g, raw, T in zip(pg["frames"], lp.raw, pg["T"]):
        gt = gt0 @ src.ground_truth_body(g)
        err_raw.append(np.linalg.norm((bt @ raw @ np.linalg.inv(bt))[:3, 3] - gt[:3, 3]))
        err_opt.append(np.linalg.norm((bt @ T @ np.linalg.inv(bt))[:3, 3] - gt[:3, 3]))
    # the newest keyframes (after the loop) move towards the ground truth
    assert np.mean(err_opt[-5:]) <= np.mean(err_raw[-5:]) + 1e-4, (err_raw[-5:], err_opt[-5:])
    assert max(err_opt) <= max(err_raw) and max(err_opt) < 0.06, err_opt
    print("keyframe position error vs ground truth: raw max %.4f m, optimised max %.4f m, last-5 %.4f -> %.4f m"
          % (max(err_raw), max(err_opt), np.mean(err_raw[-5:]), np.mean(err_opt[-5:])))
    kfs = eng.get_map().keyframe_poses
    assert len(kfs) == len(pg["frames"])
    eng.shutdown()


def _rig_loop_sources():
    import json
    from pathlib import Path

    from thor_slam_amd.synthetic import RoomScene

    mats = json.loads((Path(__file__).parent / "golden" / "brackets_joints.json").read_text())
    scene, traj = RoomScene(seed=0), circle_trajectory(LOOP_FRAMES, yaw_rate_deg=YAW)
    names = ("192.168.2.21", "192.168.2.25")
    return [SyntheticStereoSource(name=nm, scene=scene, trajectory=traj, rig_T_source=np.array(mats[nm]), seed=k)
            for k, nm in enumerate(names)], mats


def _render_rig(idx):
    srcs, _ = _rig_loop_sources()
    return [np.stack([s.render_image(i, c) for s in srcs for c in (0, 1)]) for i in idx]


def _check_loop_edges(pg, bt, src):
    """Every loop edge's measurement (T_a^-1 T_b of pair 0's rect-left camera, whichever pairs
    recognised and verified the place) against the rendered ground truth."""
    n = 0
    for (a, b), Z in zip(pg["edges"], pg["meas"]):
        if b == a + 1:
            continue
        fa, fb = pg["frames"][a], pg["frames"][b]
        gt = np.linalg.inv(bt) @ np.linalg.inv(src.ground_truth_body(fa)) @ src.ground_truth_body(fb) @ bt
        assert np.linalg.norm(Z[:3, 3] - gt[:3, 3]) < 0.03, (fa, fb, Z[:3, 3], gt[:3, 3])
        ang = np.degrees(np.arccos(np.clip((np.trace(Z[:3, :3] @ gt[:3, :3].T) - 1) / 2, -1, 1)))
        assert ang < 0.5, (fa, fb, ang)
        n += 1
    return n


def test_engine_closes_the_loop_on_a_two_source_rig():
    """The bracket rig's two stereo sources on the loop trajectory: the rig pose (k_rig_pose) is
    tracked, place recognition and verification run on pair 0's camera, and the pose graph over
    pair 0's keyframe poses taken from the body poses pulls them towards the ground truth."""
    import torch

    from thor_slam_amd.slam.hip_engine import HipSlamEngine

    srcs, mats = _rig_loop_sources()
    idx = list(range(LOOP_FRAMES))
    chunks = [idx[i::16] for i in range(16)]
    out = {}
    with ProcessPoolExecutor(max_workers=16) as ex:
        for c, frs in zip(chunks, ex.map(_render_rig, chunks)):
            out.update(zip(c, frs))
    frames = np.stack([out[i] for i in idx])
    rig = CameraRig(srcs, rig_extrinsics={s.name: Extrinsics.from_4x4_matrix(np.array(mats[s.name])) for s in srcs})
    cfg = HipSlamConfig(batch_size=30, enable_loop_closure=True)
    eng = HipSlamEngine(num_cameras=4, config=cfg)
    eng.initialize(rig.calibration, cfg)
    assert len(eng._pairs) == 2 and eng._loop is not None
    dev = torch.from_numpy(frames).cuda()
    for b0 in range(0, LOOP_FRAMES, 30):
        eng.process_batch(dev[b0:b0 + 30], [srcs[0].timestamp(i) for i in range(b0, b0 + 30)])
    eng.settle()
    loops = eng.loop_closures
    assert loops, "no loop closed"
    pg, lp, bt = eng.pose_graph, eng._loop, eng._base_T_rect
    # rig-wide recognition: besides the same-pair loops after the full turn (frame >= 225), pair
    # 1 sees pair 0's early view part-way round (and pair 0 pair 1's) -- every edge must agree
    # with the ground truth
    assert _check_loop_edges(pg, bt, srcs[0]) == len(loops)
    assert any(c <= 40 and q >= 225 and p == r for (c, q, _), (p, r) in zip(loops, lp.pairs)), (loops, lp.pairs)
    gt0 = np.linalg.inv(srcs[0].ground_truth_body(0))
    err_raw, err_opt = [], []
    for g, raw, T in zip(pg["frames"], lp.raw, pg["T"]):
        gt = gt0 @ srcs[0].ground_truth_body(g)
        err_raw.append(np.linalg.norm((bt @ raw @ np.linalg.inv(bt))[:3, 3] - gt[:3, 3]))
        err_opt.append(np.linalg.norm((bt @ T @ np.linalg.inv(bt))[:3, 3] - gt[:3, 3]))
    assert np.mean(err_opt[-5:]) <= np.mean(err_raw[-5:]) + 1e-4, (err_raw[-5:], err_opt[-5:])
    # the rig's raw drift is millimetres here, so the cross-pair loop edges (each within 3 cm /
    # 0.5 deg of the truth) may spread a few millimetres over the graph
    assert max(err_opt) < 0.03, (max(err_raw), max(err_opt))
    print("rig loops %s (pairs %s); keyframe position error vs ground truth: raw max %.4f m, optimised max %.4f m, "
          "last-5 %.4f -> %.4f m" % (loops, lp.pairs, max(err_raw), max(err_opt), np.mean(err_raw[-5:]),
                                     np.mean(err_opt[-5:])))
    eng.shutdown()


def test_rig_loop_seen_only_by_pair_1():
    """Rig-wide place recognition: pair 0 of the bracket rig is blind (flat images) for the whole
    run, so only pair 1's keyframe entries can recognise the place; the loop is found, verified on
    pair 1's camera, and its edge (moved into pair 0's frame through the rig extrinsics) agrees
    with the ground-truth relative motion of pair 0's rectified-left camera."""
    import torch

    from thor_slam_amd.slam.hip_engine import HipSlamEngine

    srcs, mats = _rig_loop_sources()
    idx = list(range(LOOP_FRAMES))
    chunks = [idx[i::16] for i in range(16)]
    out = {}
    with ProcessPoolExecutor(max_workers=16) as ex:
        for c, frs in zip(chunks, ex.map(_render_rig, chunks)):
            out.update(zip(c, frs))
    frames = np.stack([out[i] for i in idx])
    frames[:, 0:2] = 128                      # pair 0 blind
    rig = CameraRig(srcs, rig_extrinsics={s.name: Extrinsics.from_4x4_matrix(np.array(mats[s.name])) for s in srcs})
    cfg = HipSlamConfig(batch_size=30, enable_loop_closure=True)
    eng = HipSlamEngine(num_cameras=4, config=cfg)
    eng.initialize(rig.calibration, cfg)
    dev = torch.from_numpy(frames).cuda()
    for b0 in range(0, LOOP_FRAMES, 30):
        eng.process_batch(dev[b0:b0 + 30], [srcs[0].timestamp(i) for i in range(b0, b0 + 30)])
    eng.settle()
    loops = eng.loop_closures
    assert loops, "no loop closed"
    assert all(c <= 40 and q >= 225 for c, q, _ in loops), loops
    lp, bt = eng._loop, eng._base_T_rect
    assert lp.pairs and all(pq == (1, 1) for pq in lp.pairs), lp.pairs
    pg = eng.pose_graph
    _check_loop_edges(pg, bt, srcs[0])
    gt0 = np.linalg.inv(srcs[0].ground_truth_body(0))
    err_raw, err_opt = [], []
    for g, raw, T in zip(pg["frames"], lp.raw, pg["T"]):
        gt = gt0 @ srcs[0].ground_truth_body(g)
        err_raw.append(np.linalg.norm((bt @ raw @ np.linalg.inv(bt))[:3, 3] - gt[:3, 3]))
        err_opt.append(np.linalg.norm((bt @ T @ np.linalg.inv(bt))[:3, 3] - gt[:3, 3]))
    assert np.mean(err_opt[-5:]) <= np.mean(err_raw[-5:]) + 1e-4, (err_raw[-5:], err_opt[-5:])
    print("pair-1-only loop: %s; keyframe error raw max %.4f m, optimised max %.4f m"
          % (loops, max(err_raw), max(err_opt)))
    eng.shutdown()


def test_growing_pose_graph_jobs_without_polling():
    """a small pose-graph job, then larger ones, submitted back to back without a poll
    in between — the scratch grows under the queued jobs (the reserve drains the loop worker and
    stream first) — and every job returns the oracle's solve."""
    from thor_slam_amd._lib import Handle

    h = Handle([_rect(_loop_source())], HipSlamConfig(), max_batch=1)
    graphs, jobs = [], []
    for N, loops in ((6, [(0, 5)]), (40, [(0, 39), (5, 30)]), (120, [(0, 119), (7, 80), (40, 100)])):
        g = _random_graph(np.random.default_rng(N), N, loops)
        graphs.append(g)
        jobs.append(h.loop_job_pose_graph(*g, 5))
    for g, job in zip(graphs, jobs):
        got = job.result(block=True)
        want = L.optimize(*g, 5)
        assert max(rel_frobenius(a, b) for a, b in zip(got["T"], want["T"])) < 1e-9
    h.close()
