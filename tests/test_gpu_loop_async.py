"""Asynchronous loop closure: keyframes stored by the submit path
(``tslam_loop_auto``), searches as jobs on the handle's loop stream (``tslam_loop_job_*``), and
the engine's policy against ``oracle/numpy_loop.py`` ``LoopPolicy``:

* the in-stream store gives the entries the synchronous store gives (bit-identical), only for
  tracked keyframes, at consecutive database positions;
* vote / verify / pose-graph jobs equal the synchronous calls bit for bit, and the votes equal
  ``numpy_loop.vote`` on the stored descriptors;
* the reference's default drop-in path (``HipSlamEngine(num_cameras=2)`` + ``initialize`` with no
  config: batch 1, loop closure on) publishes, frame for frame, the poses ``LoopPolicy`` defines
  from the same tracked poses and search results, with its solves checked against the oracle's
  Gauss-Newton;
* a 6,000-frame session (25 laps of the loop) keeps searching after the database ring wrapped,
  and the late loops are closed as the policy defines."""

from __future__ import annotations

import numpy as np
import pytest

from test_gpu_loop import LOOP_FRAMES, _loop_source, _rect, _render_many
from oracle import numpy_loop as L
from thor_slam_amd.camera import CameraRig
from thor_slam_amd.params import HipSlamConfig

pytestmark = pytest.mark.gpu

LAP = 240   # the circle closes at frame 240 (test_gpu_loop.LOOP_FRAMES)


class _FrameReplay:
    """A CameraSource serving pre-rendered [left, right] frames in order (frame i -> frames[i % n]),
    30 fps timestamps; no IMU (the rig then names an identity IMU that sends nothing)."""

    def __init__(self, src, frames):
        self.src, self.frames, self.i = src, frames, 0

    @property
    def name(self):
        return self.src.name

    def start(self):
        pass

    def stop(self):
        pass

    def get_latest_frames(self):
        from thor_slam_amd.camera.types import CameraFrame

        k = self.i % len(self.frames)
        ts = 100.0 + self.i / 30.0
        self.i += 1
        return [CameraFrame(image=self.frames[k, c], timestamp=ts, sequence_num=self.i, camera_name=f"{self.name}_{c}")
                for c in (0, 1)]

    def try_get_latest_frames(self):
        return self.get_latest_frames()

    def get_intrinsics(self):
        return self.src.get_intrinsics()

    def get_extrinsics(self):
        return self.src.get_extrinsics()

    def get_sensor_extrinsics(self):
        return None

    def get_timestamped_sensor_data(self):
        return None, None

    def try_get_timestamped_sensor_data(self):
        return None, None

    @property
    def has_sensor_data(self):
        return False


def _lap_frames():
    return _render_many(list(range(LAP)))


def test_loop_jobs_equal_synchronous_calls():
    """Consecutive frames of the loop in batches of 30: the auto store (tracked keyframes only,
    positions 0, 1, ...) equals the manual store of the same frames; votes, verification and a
    pose-graph solve as jobs equal the synchronous calls, and the votes equal the oracle's."""
    import torch

    from thor_slam_amd._lib import Handle

    src = _loop_source()
    rect = _rect(src)
    frames = _render_many(list(range(LOOP_FRAMES)))
    n = LOOP_FRAMES
    cfg = HipSlamConfig()
    dev = torch.from_numpy(np.ascontiguousarray(frames)).cuda()
    s = torch.cuda.current_stream().cuda_stream
    auto, man = Handle([rect], cfg, max_batch=30), Handle([rect], cfg, max_batch=30)
    auto.loop_init(64, 256)
    man.loop_init(64, 256)
    auto.loop_auto(5)
    stats, pos = [], 0
    for b0 in range(0, n, 30):
        for h in (auto, man):
            h.submit(dev[b0:].data_ptr(), 30, s)
        st = auto.read_poses(30)["stats"][:, 0, 0]
        np.testing.assert_array_equal(st, man.read_poses(30)["stats"][:, 0, 0])
        stats.append(st)
        for k in range(30):   # the manual store of the same keyframes (resident in the ring)
            g = b0 + k
            if g % 5 == 0 and st[k] == 0:
                slot, _ = man.loop_add_keyframe(g)
                assert slot == pos
                pos += 1
    stats = np.concatenate(stats)
    tracked = [g for g in range(0, n, 5) if stats[g] == 0]
    assert len(tracked) == pos >= 50 and stats[0] == 2   # frame 0 (INIT) takes no position
    for e in range(pos):
        a, m = auto.loop_read_keyframe(e), man.loop_read_keyframe(e)
        assert a["xyz"].shape[0] > 500
        np.testing.assert_array_equal(a["xyz"], m["xyz"])
        np.testing.assert_array_equal(a["desc"], m["desc"])
    assert auto.loop_read_keyframe(pos)["xyz"].shape[0] == 0   # nothing past the last position
    # votes: frame 245 (the start's place again) against positions [0, 20), and a window that
    # starts mid-database against the synchronous query's slice
    q = tracked.index(245)
    job = auto.loop_job_vote(q, 0, 20)
    votes = job.result(block=True)
    np.testing.assert_array_equal(votes, auto.loop_query(q, 20))
    np.testing.assert_array_equal(auto.loop_job_vote(q, 3, 10).result(block=True), auto.loop_query(q, 13)[3:])
    descs = [auto.loop_read_keyframe(e)["desc"] for e in range(pos)]
    want = [L.vote(descs[q], descs[c], 256, cfg.max_hamming, cfg.ratio_pct) for c in range(20)]
    np.testing.assert_array_equal(votes, want)
    assert job.result() is votes   # cached by the binding
    best, _, j = L.best_vote([votes], 1)
    assert best >= cfg.loop_min_votes and tracked[j] <= 15, (best, j)
    # verification from the entry's snapshot == the synchronous one on the resident frame
    g = tracked[q]
    assert g >= n - 60   # still in the ring
    vj = auto.loop_job_verify(g, q, j).result(block=True)
    vs = auto.loop_verify(g, j)
    np.testing.assert_array_equal(vj["stats"], vs["stats"])
    np.testing.assert_array_equal(vj["T"], vs["T"])
    np.testing.assert_array_equal(vj["cov"], vs["cov"])
    assert vj["stats"][0] == 0 and vj["stats"][2] >= cfg.loop_min_inliers
    # a pose-graph job == the synchronous solve (the same kernels on the loop stream)
    rng = np.random.default_rng(3)
    T0 = [np.eye(4)]
    for _ in range(29):
        T0.append(T0[-1] @ L.se3_exp(np.r_[rng.normal(0, 0.1, 3), rng.normal(0, 0.05, 3)]))
    edges = np.array([(i, i + 1) for i in range(29)] + [(0, 29), (3, 20)])
    Z = np.stack([L.inv_se3(T0[a]) @ T0[b] @ L.se3_exp(rng.normal(0, 0.003, 6)) for a, b in edges])
    info = np.stack([L.loop_information(0.01, 0.005)] * len(edges))
    pj = auto.loop_job_pose_graph(np.stack(T0), edges, Z, info, 6).result(block=True)
    ps = auto.pose_graph(np.stack(T0), edges, Z, info, 6)
    np.testing.assert_array_equal(pj["T"], ps["T"])
    assert pj["cost"] == ps["cost"]
    ora = L.optimize(np.stack(T0), edges, Z, info, 6)
    assert max(np.linalg.norm(a - b) / np.linalg.norm(b) for a, b in zip(pj["T"], ora["T"])) < 1e-9
    # a job's results are returned once: polling its id again is refused (TSLAM_ESTATE)
    assert auto.lib.tslam_loop_job_poll(auto.h, job.id, 1, None, None, None, None, None, None) == -4
    auto.close()
    man.close()


def _run_default(frames, n_frames, settle=False, hook=None):
    """The reference's default drop-in construction (scripts/run_slam.py:299-300 after the swap):
    HipSlamEngine(num_cameras=2) + initialize(rig.calibration), no config — batch 1, loop closure
    on (SlamConfig.enable_loop_closure), the rig's identity IMU idle.  Returns per frame the
    published world_T_base (None when lost), the tracked batch records, the engine."""
    from thor_slam_amd.slam.hip_engine import HipSlamEngine

    src = _loop_source()
    rig = CameraRig([_FrameReplay(src, frames)])
    rig.start()
    eng = HipSlamEngine(num_cameras=2)
    eng.initialize(rig.calibration)
    assert eng._config.batch_size == 1 and eng._config.enable_loop_closure and eng._async
    eng._loop.trace = {}
    if hook is not None:
        hook(eng)
    recs, published = [], {}
    orig = eng._publish

    def record(res, stamps, g0):
        recs.append((g0, res["T_abs"][:len(stamps), 0].copy(), res["stats"][:len(stamps), 0, 0].copy()))
        orig(res, stamps, g0)
        p = eng._latest_pose
        published[g0 + len(stamps) - 1] = None if p is None else p.to_4x4_matrix()

    eng._publish = record
    for _ in range(n_frames):
        eng.process_frames(rig.get_synchronized_frames())
    if settle:
        eng.settle()
    else:
        eng.flush()
    return published, recs, eng


def _policy_from_trace(eng, recs, solve_check_every=0, finish=False):
    """oracle LoopPolicy on the engine's tracked poses, with the device's votes / verifications
    (the trace) and — for the solves — the device's results after asserting the policy built the
    same inputs (every ``solve_check_every``-th solve, and the last, re-solved by the oracle's
    Gauss-Newton: within 1e-9)."""
    from thor_slam_amd.slam.hip_engine import _invert

    cfg, tr = eng._config, eng._loop.trace
    checked = []

    def vote(idx, q, lo, n):
        tlo, tn, v = tr[("vote", idx, q)]
        assert (tlo, tn) == (lo, n)
        return v

    def verify(idx, g, q, c, pc):
        tq, tc, tpc, ver = tr[("verify", idx)]
        assert (tq, tc, tpc) == (q, c, pc)
        return ver

    solves = sorted(k[1] for k in tr if k[0] == "solve")
    state = {"i": 0}

    def solve(T, edges, meas, info, iters):
        idx = solves[state["i"]]
        state["i"] += 1
        (t_in, e_in, m_in, i_in), sol = tr[("solve", idx)]
        np.testing.assert_array_equal(T, t_in)
        np.testing.assert_array_equal(edges, e_in)
        np.testing.assert_array_equal(meas, m_in)
        if sol is None:   # the device rejected this span solve (TSLAM_ESINGULAR)
            raise L.SpanSolveFailed(str(idx))
        if (solve_check_every and state["i"] % solve_check_every == 1) or state["i"] == len(solves) or len(solves) < 8:
            ora = L.optimize(T, edges, meas, info, iters)
            err = max(np.linalg.norm(a - b) / np.linalg.norm(b) for a, b in zip(sol["T"], ora["T"]))
            assert err < 1e-9, (idx, err)
            checked.append(idx)
        return sol

    pol = L.LoopPolicy(cfg, 1, [np.eye(4)], vote, verify, solve)
    bt = eng._base_T_rect
    out = {}
    for g0, T_abs, st in recs:
        for k in range(len(st)):
            body = bt @ T_abs[k] @ _invert(bt)
            raw = _invert(bt) @ body @ bt   # the engine's rect-left pose before loop correction
            corr = pol.step(g0 + k, int(st[k]), raw)
            out[g0 + k] = None if pol.state != "tracking" else bt @ corr @ _invert(bt)
    if finish:   # HipSlamEngine.settle
        pol.finish()
    return pol, out, checked


def _compare(published, want, n):
    worst = 0.0
    for g in range(n):
        a, b = published.get(g), want.get(g)
        if a is None or b is None:
            assert (a is None) == (b is None), g
            continue
        worst = max(worst, float(np.linalg.norm(a[:3, 3] - b[:3, 3])),
                    float(np.linalg.norm(a[:3, :3] - b[:3, :3])))
    assert worst < 1e-9, worst
    return worst


def test_default_path_equals_loop_policy():
    """The default configuration at batch 1 over the 270-frame loop: every published pose equals
    the oracle LoopPolicy's sequence (loop_latency 30: the late loops' corrections apply 30 frames
    after their keyframes), the loop back to the start is found and closed, and process_frames
    never waited for a search of its own (searches ran as jobs)."""
    frames = _render_many(list(range(LOOP_FRAMES)))
    published, recs, eng = _run_default(frames, LOOP_FRAMES)
    pol, want, checked = _policy_from_trace(eng, recs)
    _compare(published, want, LOOP_FRAMES)
    lp = eng._loop
    assert lp.loops and lp.loops == pol.loops, (lp.loops, pol.loops)
    assert any(c <= 40 and q >= 225 for c, q, _ in lp.loops), lp.loops
    assert len(lp.frames) == len(pol.frames) and all(np.array_equal(a, b) for a, b in zip(lp.raw, pol.raw))
    # the corrections arrive loop_latency frames after their keyframe: the first loop's keyframe
    # is published uncorrected and its correction is in place from keyframe + 30 on
    g = lp.loops[0][1]
    assert g + 30 < LOOP_FRAMES and checked
    eng.shutdown()


@pytest.mark.slow
def test_long_session_keeps_closing_loops():
    """6,100 frames = 25 laps of the loop at batch 1 (default configuration): more tracked
    keyframes than the database holds (1,024), so its ring wraps, and the searches keep finding
    the previous lap: a loop with its keyframe past frame 6,000 is detected, verified and closed,
    every published pose equals LoopPolicy's, and every span solve stays within the ring."""
    frames = _lap_frames()
    n = 6100   # a loop at keyframe 6,000+ is applied loop_latency frames later
    published, recs, eng = _run_default(frames, n)
    lp = eng._loop
    assert len(lp.frames) > 1100   # > 1,024 database positions: the ring wrapped
    late = [(c, q) for c, q, _ in lp.loops if q >= 6000]
    assert late, lp.loops[-3:]
    assert all(q - c <= 5 * 1024 for c, q, _ in lp.loops)
    pol, want, checked = _policy_from_trace(eng, recs, solve_check_every=17)
    assert lp.loops == pol.loops and len(checked) >= 10
    _compare(published, want, n)
    eng.shutdown()


def test_rejected_loop_solve_keeps_the_session_running():
    """the first loop's span solve is handed an uninformative span (every
    edge's information zeroed — every direction of the span is a free gauge, the normal matrix is
    0).  The device's Cholesky fails (TSLAM_ESINGULAR) where the oracle's does (LinAlgError); the
    engine rejects that loop as LoopPolicy defines — no edge, no correction, the cooldown not
    armed — and process_frames keeps returning poses: every published pose equals the policy's,
    and the next keyframe's loop is closed."""
    frames = _render_many(list(range(LOOP_FRAMES)))
    zeroed = []

    def hook(eng):
        h = eng._loop.h
        orig = h.loop_job_pose_graph

        def degenerate_first(T, edges, meas, info, iters):
            if not zeroed:
                info = np.zeros_like(info)
                zeroed.append((np.array(T), np.array(edges), np.array(meas), info))
            return orig(T, edges, meas, info, iters)

        h.loop_job_pose_graph = degenerate_first

    # settle: the searches still pending at the end (the keyframes after the rejected one) complete
    published, recs, eng = _run_default(frames, LOOP_FRAMES, settle=True, hook=hook)
    assert zeroed
    with pytest.raises(np.linalg.LinAlgError):   # the oracle fails the same span
        L.optimize(*zeroed[0], eng._config.pg_iters)
    lp = eng._loop
    pol, want, _ = _policy_from_trace(eng, recs, finish=True)
    assert len(lp.rejected) == 1 and lp.rejected == pol.rejected, (lp.rejected, pol.rejected)
    assert "not positive definite" in lp.failures[0]["error"]
    assert lp.loops and lp.loops == pol.loops
    assert lp.loops[0][1] > lp.rejected[0][1]   # a later keyframe closed its loop
    a_node, b_node = (lp.frames.index(f) for f in lp.rejected[0])
    assert (a_node, b_node) not in lp.edges
    _compare(published, want, LOOP_FRAMES)
    assert sum(p is not None for p in published.values()) >= LOOP_FRAMES - 2
    eng.shutdown()


def test_relocalisation_after_a_blank_gap():
    """20 blank frames (a covered lens) in the reference's default drop-in
    path.  The device reports LOST through the gap (and for the first frame after it); the third
    LOST frame moves the engine to RELOCALIZING (published pose None, get_tracking_state
    RELOCALIZING); the tracked keyframes after the gap search the keyframes from before it until
    one is verified; then tracking resumes in the map's frame.  Every published pose and state
    equals oracle LoopPolicy's on the same tracked poses and search results, and after the
    relocalisation the poses are back on the gap-free run's (the gap's 30 degrees of motion,
    which the device's chain misses, are recovered)."""
    from thor_slam_amd.slam.interface import TrackingState

    frames = _render_many(list(range(LOOP_FRAMES)))
    gap = frames.copy()
    gap[100:120] = 0
    states = {}

    def hook(eng):
        orig = eng._publish

        def record(res, stamps, g0):
            orig(res, stamps, g0)
            states[g0 + len(stamps) - 1] = eng.get_tracking_state()

        eng._publish = record

    published, recs, eng = _run_default(gap, LOOP_FRAMES, hook=hook)
    lp = eng._loop
    pol, want, _ = _policy_from_trace(eng, recs)
    stats = np.concatenate([r[2] for r in recs])
    assert (stats[100:121] == 1).all() and stats[121] == 0
    assert lp.relocs and lp.relocs == pol.relocs, (lp.relocs, pol.relocs)
    _compare(published, want, LOOP_FRAMES)
    g_rel = lp.relocs[0][1]
    back = g_rel + eng._config.reloc_latency
    assert states[100] == TrackingState.LOST and states[102] == TrackingState.RELOCALIZING
    assert all(published[g] is None and states[g] == TrackingState.RELOCALIZING for g in range(102, back))
    assert all(published[g] is not None and states[g] == TrackingState.TRACKING for g in range(back, LOOP_FRAMES))
    eng.shutdown()
    ref, _, eng0 = _run_default(frames, LOOP_FRAMES)   # the same lap without the gap
    eng0.shutdown()
    end = 230 if back < 225 else LOOP_FRAMES   # before the loop closures of frame 235 (they differ by run)
    err = max(np.linalg.norm(published[g][:3, 3] - ref[g][:3, 3]) for g in range(back, end))
    assert err < 0.05, err
    print(f"relocalised at frame {g_rel} against keyframe {lp.relocs[0][0]}; position error vs the gap-free "
          f"run after it: max {err:.4f} m")
