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
