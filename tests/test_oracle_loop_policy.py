"""oracle/numpy_loop.py LoopPolicy (the asynchronous loop closure HipSlamEngine follows) on
synthetic laps with scripted place recognition: the candidate window over the database ring, the
newest-first tie rule, the cooldown, the due frame of a correction and the span solve.  CPU only."""

from __future__ import annotations

import numpy as np

from oracle import numpy_loop as L
from thor_slam_amd.params import HipSlamConfig


def _lap_pose(i: int, lap: int = 100) -> np.ndarray:
    th = 2.0 * np.pi * (i % lap) / lap
    T = np.eye(4)
    T[:3, :3] = [[np.cos(th), 0.0, np.sin(th)], [0.0, 1.0, 0.0], [-np.sin(th), 0.0, np.cos(th)]]
    T[:3, 3] = [2.0 * np.sin(th), 0.0, 2.0 * (1.0 - np.cos(th))]
    return T


def _drift(i: int) -> np.ndarray:
    """Odometry that drifts: a slow yaw / translation error growing with the frame index."""
    return L.se3_exp(np.r_[1e-4 * i, 0.0, 0.0, 0.0, 2e-5 * i, 0.0])


class _Scripted:
    """Votes: a candidate at the same place of an earlier lap gets 100 votes (all other 0);
    verification returns the true relative pose; the solve is the oracle's Gauss-Newton."""

    def __init__(self, lap: int, interval: int):
        self.lap, self.I = lap, interval
        self.frames: list[int] = []   # node -> frame (tracked keyframes)
        self.votes, self.verifies, self.solves = [], [], []

    def vote(self, idx, q, lo, n):
        g = self.frames[idx]
        v = np.array([100 if (self.frames[c] - g) % self.lap == 0 else 0 for c in range(lo, lo + n)])
        self.votes.append((idx, lo, n))
        return v

    def verify(self, idx, g, q, c, pc):
        self.verifies.append((idx, c))
        T = L.inv_se3(_lap_pose(g, self.lap)) @ _lap_pose(self.frames[c], self.lap)   # cam_q_T_cam_c
        return {"T": T, "stats": np.array([0, 200, 150, 0, 0, 0, 0, 0])}

    def solve(self, T, edges, meas, info, iters):
        self.solves.append(len(T))
        return L.optimize(T, edges, meas, info, iters)


def _run(n_frames, lap=100, **cfg_items):
    cfg = HipSlamConfig(**cfg_items)
    sc = _Scripted(lap, cfg.loop_kf_interval)
    pol = L.LoopPolicy(cfg, 1, [np.eye(4)], sc.vote, sc.verify, sc.solve)
    out, raw_all = [], []
    for g in range(n_frames):
        raw = _lap_pose(g, lap) @ _drift(g)
        status = 2 if g == 0 else 0
        if status == 0 and g % cfg.loop_kf_interval == 0:
            sc.frames.append(g)
        out.append(pol.step(g, status, raw))
        raw_all.append(raw)
    return pol, sc, out, raw_all


def test_window_and_tie_rules():
    assert L.candidate_window(100, 1024, 20, 30, 1, 5) == (0, 80)
    assert L.candidate_window(2000, 1024, 20, 30, 1, 5) == (2000 - 1024 + 7, 1980)   # margin (30 + 1) // 5 + 1
    assert L.candidate_window(2000, 1024, 20, 0, 30, 5) == (2000 - 1024 + 12, 1980)
    # ties: newest position first; across query pairs the first strictly best wins
    assert L.best_vote([np.array([7, 7, 7])], 1) == (7, 0, 2)
    assert L.best_vote([np.array([1, 9, 9, 2])], 2) == (9, 0, 2)
    assert L.best_vote([np.array([5, 0]), np.array([0, 6])], 2) == (6, 1, 1)


def test_corrections_apply_at_the_due_frame_and_pull_drift_back():
    lap, latency = 100, 30
    pol, sc, out, raw = _run(260, lap=lap, loop_latency=latency, loop_cooldown=0)
    assert pol.loops, "no loop closed"
    first_g = pol.loops[0][1]
    assert first_g >= lap and (first_g - pol.loops[0][0]) % lap == 0
    # the correction is the identity before the first loop's due frame and not after it
    for g in range(first_g + latency):
        np.testing.assert_array_equal(out[g], raw[g])
    assert not np.array_equal(out[first_g + latency], raw[first_g + latency])
    # the last span solve honours its loop edge far better than the drifting odometry did (a
    # span solve only sees the edges inside its span: older loop edges that cross its start are
    # not re-balanced, the price of a bounded solve)
    (a, b), Z = pol.edges[-1], pol.meas[-1]
    assert b != a + 1
    e_raw = np.linalg.norm(L.se3_log(L.inv_se3(Z) @ L.inv_se3(pol.raw[a]) @ pol.raw[b]))
    e_opt = np.linalg.norm(L.se3_log(L.inv_se3(Z) @ L.inv_se3(pol.T[a]) @ pol.T[b]))
    assert e_opt < 0.1 * e_raw, (a, b, e_raw, e_opt)
    # every span solve covered [candidate, keyframe]: one lap of keyframes (newest candidate wins)
    assert set(sc.solves) == {lap // 5 + 1}


def test_cooldown_and_latency_zero():
    pol0, sc0, _, _ = _run(400, loop_latency=0, loop_cooldown=0)
    pol5, sc5, _, _ = _run(400, loop_latency=0, loop_cooldown=5)
    assert len(pol0.loops) > 4 * len(pol5.loops) > 0
    idx = [pol5.frames.index(q) for _, q, _ in pol5.loops]
    assert all(b - a > 5 for a, b in zip(idx, idx[1:]))
    # latency 0: the loop's own keyframe is already corrected
    assert pol0.loops[0][1] in pol0.frames


def test_ring_wrap_keeps_searching():
    """More tracked keyframes than the ring (cap 64): candidates stay inside the newest
    cap - margin positions, and loops keep closing after the wrap."""
    pol, sc, _, _ = _run(1200, loop_max_keyframes=64, loop_latency=30, loop_cooldown=0)
    assert len(pol.frames) > 200
    for idx, lo, n in sc.votes:
        assert lo >= idx - 64 + 7 and lo + n - 1 == idx - 20
    assert pol.loops[-1][1] > 1100


def degenerate_span(n: int = 4) -> tuple:
    """A span whose normal matrix is singular: a chain of ``n`` nodes whose edge measurements equal
    the poses exactly (every residual 0, so every Jacobian is the adjoint alone) and whose last
    edge carries translation information only — the last node's rotation is a free gauge
    direction, its diagonal block diag(1, 1, 1, 0, 0, 0) gives an exactly zero Cholesky pivot."""
    T = np.stack([_lap_pose(5 * i) for i in range(n)])
    edges = np.array([(i, i + 1) for i in range(n - 1)])
    Z = np.stack([L.inv_se3(T[a]) @ T[b] for a, b in edges])
    info = np.stack([L.loop_information(0.01, 0.005)] * (n - 2) + [np.diag([1.0, 1.0, 1.0, 0.0, 0.0, 0.0])])
    return T, edges, Z, info


def test_degenerate_span_fails_the_oracle_solve():
    T, edges, Z, info = degenerate_span()
    try:
        L.optimize(T, edges, Z, info, 3)
    except np.linalg.LinAlgError:
        pass
    else:
        raise AssertionError("a span with a free gauge direction solved")
    # the well-posed chain (full information everywhere) solves and stays put (zero residuals)
    ok = L.optimize(T, edges, Z, np.stack([L.loop_information(0.01, 0.005)] * len(edges)), 3)
    np.testing.assert_allclose(ok["T"], T, atol=1e-12)


def test_rejected_span_solve_leaves_poses_uncorrected_and_the_session_running():
    """A span solve that fails (LinAlgError from the oracle, SpanSolveFailed from a device
    callable) drops that loop: no edge, no correction, the cooldown not armed; the next loop is
    closed as usual, and every frame still gets a pose."""
    lap = 100
    for exc in (np.linalg.LinAlgError, L.SpanSolveFailed):
        cfg = HipSlamConfig(loop_latency=0, loop_cooldown=50)
        sc = _Scripted(lap, cfg.loop_kf_interval)
        calls = {"n": 0}

        def solve(T, edges, meas, info, iters, exc=exc):
            calls["n"] += 1
            if calls["n"] == 1:
                raise exc("normal matrix not positive definite")
            return L.optimize(T, edges, meas, info, iters)

        pol = L.LoopPolicy(cfg, 1, [np.eye(4)], sc.vote, sc.verify, solve)
        ref = L.LoopPolicy(cfg, 1, [np.eye(4)], sc.vote, sc.verify, sc.solve)
        out = []
        for g in range(260):
            raw = _lap_pose(g, lap) @ _drift(g)
            status = 2 if g == 0 else 0
            if status == 0 and g % cfg.loop_kf_interval == 0:
                sc.frames.append(g)
            out.append(pol.step(g, status, raw))
            ref.step(g, status, raw)
            if not pol.loops:
                np.testing.assert_array_equal(out[-1], raw)   # uncorrected until a loop is closed
        assert len(pol.rejected) == 1 and ref.loops and not ref.rejected
        rej_c, rej_g = pol.rejected[0]
        assert rej_g == ref.loops[0][1]   # the first loop found is the rejected one
        # the cooldown counts closed loops only: the keyframe after the rejected one closes its loop
        assert pol.loops[0][1] == rej_g + cfg.loop_kf_interval, (pol.loops[:2], rej_g)
        assert (pol.frames.index(rej_c), pol.frames.index(rej_g)) not in pol.edges
        assert len(pol.edges) == len(pol.frames) - 1 + len(pol.loops)


def test_non_finite_solution_is_rejected():
    """A solve that returns a non-finite pose (the device's NaN propagation) is rejected too."""
    cfg = HipSlamConfig(loop_latency=0, loop_cooldown=0)
    sc = _Scripted(100, cfg.loop_kf_interval)

    def solve(T, edges, meas, info, iters):
        sol = L.optimize(T, edges, meas, info, iters)
        sol["T"][-1, 0, 0] = np.nan
        return sol

    pol = L.LoopPolicy(cfg, 1, [np.eye(4)], sc.vote, sc.verify, solve)
    for g in range(160):
        raw = _lap_pose(g, 100) @ _drift(g)
        if g and g % cfg.loop_kf_interval == 0:
            sc.frames.append(g)
        np.testing.assert_array_equal(pol.step(g, 2 if g == 0 else 0, raw), raw)
    assert pol.rejected and not pol.loops


def _run_gap(gap=(150, 170), after=3, n_frames=260, lap=100, **cfg_items):
    """A drift-free lap sequence whose frames in [gap) are LOST; the device's chain then misses the
    gap's motion, so every raw pose after it is off by the rigid error E = raw_{g0-1} raw_{g1-1}^-1
    (the LOST frames keep the last tracked pose, the first frame after the gap chains from it)."""
    cfg = HipSlamConfig(reloc_after_lost=after, **cfg_items)
    sc = _Scripted(lap, cfg.loop_kf_interval)
    pol = L.LoopPolicy(cfg, 1, [np.eye(4)], sc.vote, sc.verify, sc.solve)
    g0, g1 = gap
    E = _lap_pose(g0 - 1, lap) @ L.inv_se3(_lap_pose(g1, lap))   # first frame after the gap is LOST too
    out, states = [], []
    for g in range(n_frames):
        if g0 <= g <= g1:
            status, raw = 1, _lap_pose(g0 - 1, lap)
        else:
            status = 2 if g == 0 else 0
            raw = _lap_pose(g, lap) if g < g0 else E @ _lap_pose(g, lap)
        if status == 0 and g % cfg.loop_kf_interval == 0:
            sc.frames.append(g)
        out.append(pol.step(g, status, raw))
        states.append(pol.state)
    return pol, sc, out, states


def test_relocalisation_after_a_lost_run_reanchors_the_new_segment():
    """reloc_after_lost = 3: the third LOST frame breaks the graph (RELOCALIZING), the first
    tracked keyframe after the gap starts an unanchored segment without an odometry edge, its
    relocalisation item (due reloc_latency frames later) finds the place seen a lap earlier, and
    from then on the published poses are the true ones again; loop closure goes on afterwards."""
    lap, (g0, g1) = 100, (150, 170)
    pol, sc, out, states = _run_gap(loop_latency=30, loop_cooldown=0, reloc_latency=5)
    assert states[g0] == states[g0 + 1] == "lost" and states[g0 + 2] == "relocalizing"
    assert pol.relocs, "not relocalised"
    c_frame, g_rel, inl = pol.relocs[0]
    assert g_rel == 175 and (g_rel - c_frame) % lap == 0 and inl == 150   # the first keyframe after the gap
    first_back = g_rel + 5   # its item is due reloc_latency frames later
    assert all(s_ == "relocalizing" for s_ in states[g0 + 2:first_back])
    assert all(s_ == "tracking" for s_ in states[first_back:])
    for g in range(first_back, 260):   # the drift-free sequence: exact poses again
        np.testing.assert_allclose(out[g], _lap_pose(g, lap), atol=1e-9)
    # the segment's first node has no odometry edge to the node before the gap; the
    # relocalisation edge joins it to its candidate
    idx = pol.frames.index(g_rel)
    assert (idx - 1, idx) not in pol.edges and (pol.frames.index(c_frame), idx) in pol.edges
    assert pol.loops and pol.loops[-1][1] > first_back   # loop closure afterwards


def test_short_lost_run_and_reloc_off_do_not_break_the_graph():
    # a LOST run shorter than reloc_after_lost: no episode, the offset stays (the device's chain)
    pol, _, out, states = _run_gap(gap=(150, 151), after=3, loop_latency=30, loop_cooldown=0)
    assert "relocalizing" not in states and not pol.relocs
    # relocalisation off: the 21-frame gap leaves the later poses off by its motion
    pol0, _, out0, states0 = _run_gap(after=0, loop_latency=30, loop_cooldown=0)
    assert "relocalizing" not in states0 and not pol0.relocs
    assert np.abs(out0[200][:3, 3] - _lap_pose(200)[:3, 3]).max() > 0.1
