"""CPU checks of the A8 oracle (oracle/numpy_ba.py): the spec the HIP BA kernels are tested against.

cuVSLAM's BA is closed, so these pin the restatement by properties: exact
observations converge to the true poses, eviction keeps every landmark homed in an occupied slot
that observes it, and chained temporal maps compose.
"""

from __future__ import annotations

import numpy as np

from oracle.numpy_ba import BAParams, BATracker, KeyframeWindow, chain_links
from oracle.numpy_slam import cayley

FX, FY, CX, CY, BASE = 384.0, 384.0, 319.5, 199.5, 0.075


def _world(K: int, rng) -> np.ndarray:
    return np.stack([rng.uniform(-2, 2, K), rng.uniform(-1, 1, K), rng.uniform(3, 6, K)], 1)


def _cam(j: int) -> np.ndarray:
    T = np.eye(4)
    T[:3, :3] = cayley(np.array([0.0, 0.02 * j, 0.0]))
    T[:3, 3] = [-0.05 * j, 0.0, 0.0]
    return T


def _observe(T: np.ndarray, Pw: np.ndarray):
    xc = Pw @ T[:3, :3].T + T[:3, 3]
    return FX * xc[:, 0] / xc[:, 2] + CX, FY * xc[:, 1] / xc[:, 2] + CY, FX * BASE / xc[:, 2]


def test_exact_observations_converge():
    rng = np.random.default_rng(0)
    K = 200
    win = KeyframeWindow(K, (FX, FY, CX, CY, FX * BASE), BAParams(window=5, iters=8, lam=1e-3, outlier_px=50.0))
    Pw = _world(K, rng)
    for j in range(5):
        T = _cam(j)
        u, v, d = _observe(T, Pw)
        Tn = T.copy()
        if j:   # perturbed initial pose; keyframe 0 is the gauge
            Tn[:3, :3] = cayley(rng.normal(0, 0.01, 3)) @ T[:3, :3]
            Tn[:3, 3] += rng.normal(0, 0.01, 3)
        win.add_keyframe(5 * j, Tn, u, v, d, None if j == 0 else np.arange(K))
    res = win.solve()
    assert res["n_lm"] == K and res["n_obs"] == 5 * K
    assert res["rms_px"] < 1e-6
    for j, s in enumerate(win.order()):
        assert np.abs(win.T_cw[s] - _cam(j)).max() < 1e-8


def test_outlier_gate_and_min_observations():
    rng = np.random.default_rng(1)
    K = 50
    win = KeyframeWindow(K, (FX, FY, CX, CY, FX * BASE), BAParams(window=3, iters=2, outlier_px=3.0))
    Pw = _world(K, rng)
    for j in range(3):
        u, v, d = _observe(_cam(j), Pw)
        if j == 2:
            u = u.copy()
            u[:10] += 20.0   # 10 gross outliers in the newest keyframe
        win.add_keyframe(j, _cam(j), u, v, d, None if j == 0 else np.arange(K))
    res = win.solve()
    assert res["n_obs"] == 3 * K - 10 and res["n_lm"] == K


def test_eviction_rehomes_landmarks():
    rng = np.random.default_rng(2)
    K = 40
    W = 3
    win = KeyframeWindow(K, (FX, FY, CX, CY, FX * BASE), BAParams(window=W, iters=1))
    Pw = _world(K, rng)
    for j in range(7):
        u, v, d = _observe(_cam(j), Pw)
        link = None if j == 0 else np.where(np.arange(K) % 7 == j % 7, -1, np.arange(K))   # break some tracks
        win.add_keyframe(j, _cam(j), u, v, d, link)
        occ = win.order()
        for s in occ:
            for k in np.nonzero(win.lm[s] >= 0)[0]:
                lid = win.lm[s][k]
                home, kk = divmod(int(lid), K)
                assert home in occ and win.lm[home][kk] == lid   # homed where it is observed
        for s in range(W):
            if s not in occ:
                assert (win.lm[s] < 0).all()


def test_chain_links():
    a = np.array([2, -1, 0, 1])   # frame g -> g-1
    b = np.array([3, 0, -1, 2])   # frame g-1 -> g-2
    np.testing.assert_array_equal(chain_links([a]), a)
    np.testing.assert_array_equal(chain_links([a, b]), [-1, -1, 3, 0])


def test_tracker_composes_front_end_motion():
    """With a front end that is already exact and exact observations, keyframe poses stay put."""
    rng = np.random.default_rng(3)
    K = 60
    Pw = _world(K, rng)
    trk = BATracker(K, (FX, FY, CX, CY, FX * BASE), BAParams(window=3, kf_interval=2, iters=3))
    for g in range(9):
        T = _cam(g)
        u, v, d = _observe(T, Pw)
        kp = {"x": np.zeros(K, dtype=np.int64), "y": np.zeros(K, dtype=np.int64), "level": np.zeros(K, dtype=np.int64)}
        left = {"kp": kp, "valid": np.ones(K, dtype=bool)}
        res = {"frame": g, "world_T_cam": np.linalg.inv(T),
               "cur": {"left": left, "temporal": np.arange(K) if g else np.full(K, -1), "disp": d}}
        # level-0 coordinates are (x + 0.5) - 0.5 = x: feed the exact projections through a patched observer
        import oracle.numpy_ba as nb
        orig = nb.keyframe_observations
        nb.keyframe_observations = lambda left_, K_, u=u, v=v: (u, v)
        try:
            trk.step(res)
        finally:
            nb.keyframe_observations = orig
    w = trk.win
    assert w.n_kf == 5
    for s in w.order():
        assert np.abs(w.T_cw[s] - _cam(int(w.frame[s]))).max() < 1e-9


# -- rig-level window (all pairs' keyframes in one Schur system) ----
def _rig_E():
    """base_T_rect-left of two pairs: pair 0 forward, pair 1 turned 90 degrees about y, offset."""
    e0 = np.eye(4)
    e0[:3, 3] = [0.02, 0.0, 0.01]
    e1 = np.eye(4)
    e1[:3, :3] = np.array([[0.0, 0.0, 1.0], [0.0, 1.0, 0.0], [-1.0, 0.0, 0.0]])
    e1[:3, 3] = [0.05, -0.01, 0.0]
    return [e0, e1]


def _body(j: int) -> np.ndarray:   # body_T_world
    return _cam(j)


def test_rig_window_with_one_identity_pair_is_the_pair_window():
    from oracle.numpy_ba import RigKeyframeWindow

    rng = np.random.default_rng(4)
    K = 120
    bp = BAParams(window=4, iters=4, lam=1e-2, outlier_px=50.0)
    intr = (FX, FY, CX, CY, FX * BASE)
    one = KeyframeWindow(K, intr, bp)
    rig = RigKeyframeWindow(K, [intr], [np.eye(4)], bp)
    Pw = _world(K, rng)
    for j in range(4):
        T = _cam(j)
        u, v, d = _observe(T, Pw)
        Tn = T.copy()
        if j:
            Tn[:3, :3] = cayley(rng.normal(0, 0.01, 3)) @ T[:3, :3]
            Tn[:3, 3] += rng.normal(0, 0.01, 3)
        link = None if j == 0 else np.arange(K)
        one.add_keyframe(j, Tn, u, v, d, link)
        rig.add_keyframe(j, Tn, [(u, v, d, link)])
        a, b = one.solve(), rig.solve()
        assert a["n_obs"] == b["n_obs"] and a["n_lm"] == b["n_lm"]
        for s in one.order():
            assert np.abs(one.T_cw[s] - rig.pairs[0].T_cw[s]).max() < 1e-12
            assert np.abs(rig.B[s] - rig.pairs[0].T_cw[s]).max() < 1e-12
        np.testing.assert_allclose(rig.pairs[0].X, one.X, rtol=0, atol=1e-12)


def test_rig_window_exact_observations_converge_to_the_bodies():
    """Two pairs looking in different directions, exact observations, perturbed body poses: the
    joint solve recovers every body pose and keeps each pair's cameras at E_p^-1 B."""
    from oracle.numpy_ba import RigKeyframeWindow
    from oracle.numpy_rig import inv_rigid

    rng = np.random.default_rng(5)
    K = 150
    E = _rig_E()
    intr = (FX, FY, CX, CY, FX * BASE)
    rig = RigKeyframeWindow(K, [intr, intr], E, BAParams(window=5, iters=8, lam=1e-3, outlier_px=80.0))
    Pw = [_world(K, rng), _world(K, rng)]
    for p in range(2):   # put each pair's points in front of it: world points seen through E_p
        Pw[p] = (Pw[p] @ E[p][:3, :3].T) + E[p][:3, 3]
    for j in range(5):
        B = _body(j)
        obs = []
        for p in range(2):
            u, v, d = _observe(inv_rigid(E[p]) @ B, Pw[p])
            obs.append((u, v, d, None if j == 0 else np.arange(K)))
        Bn = B.copy()
        if j:
            Bn[:3, :3] = cayley(rng.normal(0, 0.01, 3)) @ B[:3, :3]
            Bn[:3, 3] += rng.normal(0, 0.01, 3)
        rig.add_keyframe(5 * j, Bn, obs)
    res = rig.solve()
    assert res["n_lm"] == 2 * K and res["n_obs"] == 10 * K
    for j, s in enumerate(rig.order()):
        assert np.abs(rig.B[s] - _body(j)).max() < 1e-8
        for p in range(2):
            assert np.abs(rig.pairs[p].T_cw[s] - inv_rigid(E[p]) @ rig.B[s]).max() < 1e-12


def test_rig_window_blind_pair_keeps_the_body():
    """Pair 1 sees nothing: the rig solve equals pair 0's own window moved into the body frame."""
    from oracle.numpy_ba import RigKeyframeWindow
    from oracle.numpy_rig import inv_rigid

    rng = np.random.default_rng(6)
    K = 100
    E = _rig_E()
    intr = (FX, FY, CX, CY, FX * BASE)
    rig = RigKeyframeWindow(K, [intr, intr], E, BAParams(window=4, iters=5, lam=1e-3, outlier_px=80.0))
    Pw = (_world(K, rng) @ E[0][:3, :3].T) + E[0][:3, 3]
    nan = np.full(K, np.nan)
    for j in range(4):
        B = _body(j)
        u, v, d = _observe(inv_rigid(E[0]) @ B, Pw)
        link = None if j == 0 else np.arange(K)
        Bn = B.copy()
        if j:
            Bn[:3, 3] += rng.normal(0, 0.01, 3)
        rig.add_keyframe(j, Bn, [(u, v, d, link), (nan, nan, nan, link)])
    res = rig.solve()
    assert res["pairs"][1]["n_obs"] == 0 and res["pairs"][0]["n_lm"] == K
    for j, s in enumerate(rig.order()):
        assert np.abs(rig.B[s] - _body(j)).max() < 1e-8
