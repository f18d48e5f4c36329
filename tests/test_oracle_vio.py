"""The tightly coupled visual-inertial window of the A8 oracle (oracle/numpy_ba.py: inertial factors
with velocity, position and gyro-rotation rows, per-keyframe velocities and accelerometer /
gyroscope biases tied by random-walk factors).  CPU only.

cuVSLAM's fusion is closed, so these pin the restatement by properties: the
analytic Jacobian equals finite differences through the solver's own update, the preintegration
of the synthetic IMU vanishes at the true trajectory and its gyro-bias Jacobians predict a
re-integration with another bias, exact factors and observations converge to the true poses,
velocities and biases, a synthetic IMU with a true gyroscope bias has it recovered, and a window
without factors solves as before, bit for bit.
"""

from __future__ import annotations

import numpy as np

from oracle import numpy_ba as B
from oracle.numpy_slam import cayley
from thor_slam_amd.synthetic import DRB_TO_RDF, SyntheticStereoSource

FX, FY, CX, CY, BASE = 384.0, 384.0, 319.5, 199.5, 0.075
LEVER = np.array([0.0375, 0.0, 0.0])   # the IMU (source origin) seen from the left camera


def _rand_pose(rng) -> np.ndarray:
    T = np.eye(4)
    T[:3, :3] = cayley(rng.normal(0, 0.3, 3))
    T[:3, 3] = rng.normal(0, 1.0, 3)
    return T


def _left_update(T: np.ndarray, d: np.ndarray) -> np.ndarray:
    """The BA's camera update: R <- cayley(w) R, t <- cayley(w) t + rho."""
    ru = cayley(d[3:])
    out = np.eye(4)
    out[:3, :3] = ru @ T[:3, :3]
    out[:3, 3] = ru @ T[:3, 3] + d[:3]
    return out


def _asym(A: np.ndarray) -> np.ndarray:
    return 0.5 * np.array([A[2, 1] - A[1, 2], A[0, 2] - A[2, 0], A[1, 0] - A[0, 1]])


def test_inertial_jacobian_matches_finite_differences():
    """Every column of the 15 x 30 Jacobian against central differences of the residual (the
    rotation rows at a consistent gyro rotation, A = I, where their Q^T / -I form is exact)."""
    rng = np.random.default_rng(0)
    gw = np.array([0.3, -9.7, 1.1])
    for _ in range(5):
        Ti, Tj = _rand_pose(rng), _rand_pose(rng)
        vi, vj = rng.normal(0, 1, 3), rng.normal(0, 1, 3)
        bi, bj = rng.normal(0, 0.05, 6), rng.normal(0, 0.05, 6)
        f = np.zeros(B.INE_N)
        f[0:6] = rng.normal(0, 1, 6)
        f[6:24] = rng.normal(0, 0.1, 18)
        f[24:27] = rng.normal(0, 0.05, 3)
        f[27] = 0.17
        f[32:41] = (Tj[:3, :3] @ Ti[:3, :3].T).reshape(9)   # M = Q: A = I
        f[41:68] = rng.normal(0, 0.1, 27)
        f[68:71] = bi[3:6]   # dbg = 0 at the point (the rotation rows' e(A) is then the whole residual)

        def res(x):
            A, C = _left_update(Ti, x[0:6]), _left_update(Tj, x[6:12])
            return B.inertial_residual(f, A[:3, :3], A[:3, 3], C[:3, :3], C[:3, 3], vi + x[12:15], vj + x[21:24],
                                       bi + x[15:21], bj + x[24:30], gw)

        J = B.inertial_jacobian(f, Ti[:3, :3], Ti[:3, 3], Tj[:3, :3], Tj[:3, 3], vi, vj, gw)
        h = 1e-6
        Jn = np.stack([(res(h * e) - res(-h * e)) / (2 * h) for e in np.eye(30)], axis=1)
        np.testing.assert_allclose(J, Jn, rtol=0, atol=1e-6)


def _synthetic_window(src, ri, i0, j0, bg, ba, wp):
    dt = 1.0 / src.fps
    smp = [(dt, src.imu_sample(k)["gyroscope"] + bg, src.imu_sample(k)["accelerometer"] + ba) for k in range(i0 + 1, j0 + 1)]
    return smp, B.preintegrate(smp, ri, np.zeros(3), np.zeros(3), LEVER, w_prev=wp, gyro_density=1.0e-3,
                               acc_rw=3.0e-3, gyro_rw=2.0e-4)


def test_preintegrated_synthetic_imu_vanishes_at_the_truth():
    """The synthetic IMU (samples of the rendered trajectory, lever arm included) preintegrated
    between keyframes 5 frames apart: the factor's residual at the true camera poses and
    central-difference velocities is ~1e-5 m/s, ~1e-6 m and ~1e-6 rad (gyro rotation rows)."""
    src = SyntheticStereoSource(seed=0, imu=True, n_frames=60)
    ri = DRB_TO_RDF[:3, :3]
    dt = 1.0 / src.fps
    c0 = src.camera_pose(0, 0)
    T = [np.linalg.inv(c0) @ src.camera_pose(i, 0) for i in range(42)]   # world_T_cam, world = camera 0
    gw = c0[:3, :3].T @ np.array([0.0, 0.0, -9.81])
    pos = [t[:3, 3] for t in T]
    for i0 in (5, 10, 20, 30):
        j0 = i0 + 5
        _, f = _synthetic_window(src, ri, i0, j0, np.zeros(3), np.zeros(3), ri @ src.imu_sample(i0)["gyroscope"])
        Ti, Tj = np.linalg.inv(T[i0]), np.linalg.inv(T[j0])
        vi, vj = (pos[i0 + 1] - pos[i0 - 1]) / (2 * dt), (pos[j0 + 1] - pos[j0 - 1]) / (2 * dt)
        r = B.inertial_residual(f, Ti[:3, :3], Ti[:3, 3], Tj[:3, :3], Tj[:3, 3], vi, vj, np.zeros(6), np.zeros(6), gw)
        assert np.abs(r[:3]).max() < 1e-4 and np.abs(r[3:6]).max() < 1e-5 and np.abs(r[6:9]).max() < 1e-5, (i0, r)
        assert f[28] > 0 and f[29] > 0 and f[30] > 0 and f[31] > 0 and f[71] > 0 and abs(f[27] - 5 * dt) < 1e-12


def test_gyro_bias_jacobians_predict_a_reintegration():
    """dv, dp and the rotation residual of a record integrated with bias bg_lin, corrected to first
    order by Jvg, Jpg and JRe, match a re-integration with bg_lin + d to O(|d|^2)."""
    src = SyntheticStereoSource(seed=0, imu=True, n_frames=60)
    ri = DRB_TO_RDF[:3, :3]
    smp, f0 = _synthetic_window(src, ri, 10, 15, np.zeros(3), np.zeros(3), None)
    Q = f0[32:41].reshape(3, 3)   # any fixed camera rotation: the consistent one
    for scale in (1e-3, 2e-3):
        d = scale * np.array([1.0, -2.0, 0.5])
        f1 = B.preintegrate(smp, ri, d, np.zeros(3), LEVER)
        pred_v = f0[0:3] + f0[50:59].reshape(3, 3) @ d
        pred_p = f0[3:6] + f0[59:68].reshape(3, 3) @ d
        e1 = _asym(f1[32:41].reshape(3, 3).T @ Q)   # residual of the re-integrated rotation
        e0 = _asym(f0[32:41].reshape(3, 3).T @ Q) + f0[41:50].reshape(3, 3) @ d
        errs = (np.abs(f1[0:3] - pred_v).max(), np.abs(f1[3:6] - pred_p).max(), np.abs(e1 - e0).max())
        moves = (np.abs(f1[0:3] - f0[0:3]).max(), np.abs(f1[3:6] - f0[3:6]).max(), np.abs(e1).max())
        for err, mv in zip(errs, moves):
            assert err < 0.02 * mv + 1e-12, (scale, errs, moves)


def _world(K: int, rng) -> np.ndarray:
    return np.stack([rng.uniform(-2, 2, K), rng.uniform(-1, 1, K), rng.uniform(3, 6, K)], 1)


def _traj(j: int, dt: float):
    """cam_T_world, camera centre and world velocity of a turning, accelerating camera."""
    t = j * dt
    w = np.array([0.05, 0.4, 0.1])
    R_wc = cayley(w * t)
    p = np.array([0.3 * t + 0.2 * t * t, 0.05 * t, 0.1 * t * t])
    v = np.array([0.3 + 0.4 * t, 0.05, 0.2 * t])
    T = np.eye(4)
    T[:3, :3] = R_wc.T
    T[:3, 3] = -R_wc.T @ p
    return T, p, v


def _observe(T: np.ndarray, Pw: np.ndarray):
    xc = Pw @ T[:3, :3].T + T[:3, 3]
    return FX * xc[:, 0] / xc[:, 2] + CX, FY * xc[:, 1] / xc[:, 2] + CY, FX * BASE / xc[:, 2]


def _exact_factor(Ti, vi, Tj, vj, gw, dt, b_true, b_lin, rng) -> np.ndarray:
    """A factor record whose residual vanishes at the true state (cameras, velocities, biases
    b = (ba, bg), constant over the window)."""
    f = np.zeros(B.INE_N)
    Jv, Jp = rng.normal(0, 0.2, (3, 3)) * dt, rng.normal(0, 0.02, (3, 3)) * dt
    Jvg, Jpg, JRe = rng.normal(0, 0.2, (3, 3)) * dt, rng.normal(0, 0.02, (3, 3)) * dt, -np.eye(3) * dt + rng.normal(0, 0.01, (3, 3))
    dba, dbg = b_true[0:3] - b_lin[0:3], b_true[3:6] - b_lin[3:6]
    pi, pj = -Ti[:3, :3].T @ Ti[:3, 3], -Tj[:3, :3].T @ Tj[:3, 3]
    dv = Ti[:3, :3] @ (vj - vi - gw * dt) - Jv @ dba - Jvg @ dbg
    dp = Ti[:3, :3] @ (pj - pi - vi * dt - 0.5 * gw * dt * dt) - Jp @ dba - Jpg @ dbg
    t = -JRe @ dbg   # the gyro rotation: vee-asym(M^T Q) = t, i.e. M^T Q = exp(phi), sin|phi| phi / |phi| = t
    th = np.arcsin(min(np.linalg.norm(t), 1.0))
    A = B._exp_so3(t / max(np.linalg.norm(t), 1e-300) * th)
    M = (Tj[:3, :3] @ Ti[:3, :3].T) @ A.T
    f[0:3], f[3:6], f[6:15], f[15:24], f[24:27] = dv, dp, Jv.reshape(9), Jp.reshape(9), b_lin[0:3]
    f[27], f[28], f[29], f[30], f[31] = dt, 1e4, 1e6, 1e5, 1e6
    f[32:41], f[41:50], f[50:59], f[59:68], f[68:71], f[71] = M.reshape(9), JRe.reshape(9), Jvg.reshape(9), Jpg.reshape(9), b_lin[3:6], 1e6
    return f


def test_exact_window_converges_to_poses_velocities_and_biases():
    rng = np.random.default_rng(3)
    K, n, dt = 200, 5, 1.0 / 6.0
    gw = np.array([0.0, 9.81, 0.0])
    b_true, b_lin = np.array([0.04, -0.03, 0.02, 0.01, -0.02, 0.015]), np.zeros(6)
    win = B.KeyframeWindow(K, (FX, FY, CX, CY, FX * BASE), B.BAParams(window=n, iters=25, lam=1e-4, outlier_px=50.0))
    win.set_inertial(gw, np.zeros(3), 1e-9, np.zeros(3), 1e-9)   # priors too weak to move the optimum
    Pw = _world(K, rng)
    truth = [_traj(j, dt) for j in range(n)]
    for j in range(n):
        T, _, v = truth[j]
        u, vv, d = _observe(T, Pw)
        Tn = T.copy()
        if j:
            Tn[:3, :3] = cayley(rng.normal(0, 0.01, 3)) @ T[:3, :3]
            Tn[:3, 3] += rng.normal(0, 0.01, 3)
        ine = None if j == 0 else (_exact_factor(truth[j - 1][0], truth[j - 1][2], T, v, gw, dt, b_true, b_lin, rng),
                                   v + rng.normal(0, 0.1, 3))
        win.add_keyframe(5 * j, Tn, u, vv, d, None if j == 0 else np.arange(K), ine=ine)
    win.vel[win.order()[0]] = truth[0][2] + 0.1   # the oldest keyframe's velocity: wrong too
    res = win.solve()
    assert res["rms_px"] < 1e-6
    for j, s in enumerate(win.order()):
        assert np.abs(win.T_cw[s] - truth[j][0]).max() < 1e-8
        np.testing.assert_allclose(win.vel[s], truth[j][2], atol=1e-6)
        if j < n - 1:   # the newest keyframe's biases are tied by the random walk only
            np.testing.assert_allclose(win.bias[s], b_true, atol=1e-5)


def test_true_gyro_bias_is_recovered_from_the_synthetic_imu():
    """The synthetic IMU with a true gyroscope bias of (0.02, -0.015, 0.01) rad/s, preintegrated
    at bg_lin = 0 over 5-frame keyframe intervals, in a window whose cameras see exact landmarks of
    the true trajectory: every keyframe's estimated gyroscope bias lands on the truth (within
    the preintegration's own discretisation error), where it started at zero."""
    src = SyntheticStereoSource(seed=0, imu=True, n_frames=60)
    ri = DRB_TO_RDF[:3, :3]
    bg_true = np.array([0.02, -0.015, 0.01])
    dt = 1.0 / src.fps
    c0 = src.camera_pose(0, 0)
    Tw = [np.linalg.inv(c0) @ src.camera_pose(i, 0) for i in range(42)]
    gw = c0[:3, :3].T @ np.array([0.0, 0.0, -9.81])
    rng = np.random.default_rng(7)
    K, n, iv = 150, 6, 5
    win = B.KeyframeWindow(K, (FX, FY, CX, CY, FX * BASE), B.BAParams(window=n, iters=10, lam=1e-3, outlier_px=50.0))
    win.set_inertial(gw, np.zeros(3), 1e-6, np.zeros(3), 1e-6)
    Pw = np.stack([rng.uniform(-3, 3, K), rng.uniform(-2, 2, K), rng.uniform(2, 6, K)], 1)
    for j in range(n):
        g = 5 + iv * j
        T = np.linalg.inv(Tw[g])
        Pwc = (Pw - Pw.mean(0)) + Tw[g][:3, 3] + Tw[g][:3, :3] @ np.array([0.0, 0.0, 4.0])   # in front of camera g
        u, vv, d = _observe(T, Pwc if j == 0 else Pw_used)
        Pw_used = Pwc if j == 0 else Pw_used
        ine = None
        if j:
            g0 = g - iv
            _, f = _synthetic_window(src, ri, g0, g, bg_true, np.zeros(3), ri @ (src.imu_sample(g0)["gyroscope"] + bg_true))
            v_true = (Tw[g + 1][:3, 3] - Tw[g - 1][:3, 3]) / (2 * dt)
            ine = (f, v_true)
        win.add_keyframe(g, T, u, vv, d, None if j == 0 else np.arange(K), ine=ine)
    res = win.solve()
    assert res["n_obs"] > 0
    for j, s in enumerate(win.order()[:-1]):
        np.testing.assert_allclose(win.bias[s][3:6], bg_true, atol=2e-3)


def test_window_without_inertial_factors_is_unchanged():
    K, n = 120, 4
    out = []
    for with_cfg in (False, True):
        r2 = np.random.default_rng(5)
        win = B.KeyframeWindow(K, (FX, FY, CX, CY, FX * BASE), B.BAParams(window=n, iters=3, lam=1.0, outlier_px=50.0))
        if with_cfg:
            win.set_inertial(np.array([0.0, 9.81, 0.0]), np.ones(3), 5.0)
        Pw = _world(K, np.random.default_rng(6))
        for j in range(n):
            T, _, _ = _traj(j, 0.2)
            u, vv, d = _observe(T, Pw)
            u = u + r2.normal(0, 0.3, K)
            win.add_keyframe(5 * j, T, u, vv, d, None if j == 0 else np.arange(K))
        win.solve()
        out.append((win.T_cw.copy(), win.X.copy(), win.vel.copy(), win.bias.copy()))
    for a, b in zip(out[0], out[1]):
        np.testing.assert_array_equal(a, b)
