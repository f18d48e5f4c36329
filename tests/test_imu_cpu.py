"""IMU fusion's host side: the product filter (thor_slam_amd/imu.py) against
its spec (oracle/numpy_imu.py) with and without the accelerometer leg, the gyroscope-bias estimate,
and the synthetic IMU against the trajectory it is sampled from.  CPU only."""

import numpy as np
import pytest
from scipy.spatial.transform import Rotation

from oracle import numpy_imu as OI
from thor_slam_amd.imu import ImuNoise, ImuPropagator
from thor_slam_amd.synthetic import DRB_TO_RDF, SyntheticStereoSource


def _samples(src, n):
    out = []
    for i in range(n):
        s = src.imu_sample(i)
        out.append((None if i == 0 else 1.0 / src.fps, s["gyroscope"], s["accelerometer"]))
    return out


def _rect_R_imu(src):
    # IMU axes (DRB) -> the left camera's RDF axes (rectification is the identity here)
    return DRB_TO_RDF[:3, :3]


LEVER = np.array([0.0375, 0.0, 0.0])   # the IMU (source origin) seen from the left camera


def _pair(accel: bool):
    ri = DRB_TO_RDF[:3, :3]
    noise = ImuNoise()
    prod = ImuPropagator(ri, noise, lever=LEVER, accel=accel)
    spec = OI.ImuFilter(ri, noise.acc_density, noise.acc_random_walk, noise.gyro_density, noise.gyro_random_walk,
                        noise.rot_floor, noise.trans_floor, noise.v0_sigma, noise.ba0_sigma, noise.bg0_sigma,
                        lever=LEVER, accel=accel, vis_rot_floor=noise.vis_rot_floor)
    return prod, spec


@pytest.mark.parametrize("batch,accel", [(1, True), (4, True), (4, False)])
def test_filter_matches_oracle(batch, accel):
    """Priors and states agree over a sequence with tracked and lost frames, in the batch flow."""
    src = SyntheticStereoSource(seed=0, imu=True, gyro_noise=1e-3, accel_noise=0.02, n_frames=40,
                                gyro_bias=[2e-3, -1e-3, 3e-3])
    n = 24
    smp = _samples(src, n)
    prod, spec = _pair(accel)
    rng = np.random.default_rng(1)
    for b0 in range(0, n, batch):
        idx = list(range(b0, min(n, b0 + batch)))
        if not spec.ready:
            spec.start(smp[b0][2])
            prod.begin(smp[b0][2])
        got = prod.batch_priors([smp[i] for i in idx])
        want = OI.batch_priors(spec, [smp[i] for i in idx])
        for g, w in zip(got, want):
            assert (g is None) == (w is None)
            if g is not None:
                np.testing.assert_allclose(g.R_rel, w[0], rtol=0, atol=1e-15)
                np.testing.assert_allclose(g.t_rel, w[2], rtol=1e-12, atol=1e-15)
                assert g.w_rot == pytest.approx(w[1], rel=1e-12) and g.w_trans == pytest.approx(w[3], rel=1e-12)
        # results: the true relative motion (+ noise), some frames lost
        status = np.array([0 if (i % 7) else 1 for i in idx])
        t_rel, cov = [], []
        for i in idx:
            a, b = src.camera_pose(max(i - 1, 0), 0), src.camera_pose(i, 0)
            t = np.linalg.inv(b) @ a
            t[:3, 3] += rng.normal(0, 1e-3, 3)
            t_rel.append(t)
            cov.append(np.diag([1e-6] * 3 + [1e-8] * 3))
        prod.absorb([smp[i] for i in idx], status, np.array(t_rel), np.array(cov))
        for k, i in enumerate(idx):
            if smp[i][0] is not None:
                spec.update(spec.predict(*smp[i]), int(status[k]), t_rel[k], cov[k])
        np.testing.assert_allclose(prod.st.v, spec.v, rtol=1e-10, atol=1e-14)
        np.testing.assert_allclose(prod.st.ba, spec.ba, rtol=1e-10, atol=1e-14)
        np.testing.assert_allclose(prod.st.R, spec.R, rtol=0, atol=1e-14)
        np.testing.assert_allclose(prod.st.bg, spec.bg, rtol=1e-10, atol=1e-14)
        assert prod.st.var_v == pytest.approx(spec.var_v, rel=1e-12)
        assert prod.st.var_g == pytest.approx(spec.var_g, rel=1e-12)


def test_synthetic_imu_integrates_to_the_trajectory():
    """Coasting the filter on noise-free samples from the true initial velocity reproduces the
    rendered camera motion: the samples carry the trajectory's specific force and rotation."""
    src = SyntheticStereoSource(seed=0, imu=True, n_frames=60)
    ri = _rect_R_imu(src)
    prod = ImuPropagator(ri, ImuNoise(), lever=LEVER)
    smp = _samples(src, 31)
    prod.begin(smp[0][2])
    # world = camera 0 at frame 0; the velocity at frame 0 such that the first interval's
    # constant-acceleration step lands on frame 1
    c0 = src.camera_pose(0, 0)
    pos = [(np.linalg.inv(c0) @ src.camera_pose(i, 0))[:3, 3] for i in range(3)]
    dt = 1.0 / src.fps
    st = prod.st.copy()
    st.v = (pos[1] - pos[0]) / dt - 0.5 * (pos[2] - 2 * pos[1] + pos[0]) / dt
    p = np.zeros(3)
    for i in range(1, 31):
        s = prod.step(st, *smp[i])
        p = p + st.R @ (-(s.R_rel.T @ s.t_rel))
        st = prod.coast(st, s)
    truth = (np.linalg.inv(c0) @ src.camera_pose(30, 0))[:3, 3]
    assert np.linalg.norm(p - truth) < 2e-3
    rot_true = (np.linalg.inv(c0) @ src.camera_pose(30, 0))[:3, :3]
    rot_err = Rotation.from_matrix(st.R.T @ rot_true).magnitude()
    assert rot_err < 1e-3


def test_gyro_bias_estimate_converges():
    """A constant gyroscope bias: the filter, fed the true visual motions (with the rotation
    noise its covariance states), estimates it, and its rotation priors lose the bias."""
    bias = np.array([4e-3, -2e-3, 3e-3])   # rad/s, DRB axes
    src = SyntheticStereoSource(seed=0, imu=True, gyro_noise=1e-4, n_frames=120, gyro_bias=bias)
    n = 90
    smp = _samples(src, n)
    prod, _ = _pair(False)
    prod.begin()
    rng = np.random.default_rng(3)
    first_err = last_err = None
    for i in range(1, n):
        a, b = src.camera_pose(i - 1, 0), src.camera_pose(i, 0)
        t = np.linalg.inv(b) @ a
        s = prod.step(prod.st, *smp[i])
        err = Rotation.from_matrix(s.R_rel @ t[:3, :3].T).magnitude()
        first_err = err if first_err is None else first_err
        last_err = err
        noisy = Rotation.from_rotvec(rng.normal(0, 3e-5, 3)).as_matrix() @ t[:3, :3]
        t[:3, :3] = noisy
        prod.st = prod.correct(prod.st, s, t, np.diag([1e-6] * 3 + [(3e-5) ** 2] * 3))
    assert np.linalg.norm(prod.st.bg - bias) < 0.1 * np.linalg.norm(bias), prod.st.bg
    assert last_err < 0.2 * first_err, (first_err, last_err)


def test_vision_only_matches_oracle():
    """The native tslam_imu_vision_only against the spec's vision_only: a prior-weighted solution
    moved back to the vision alone (pose and covariance), and the pass-through cases."""
    from thor_slam_amd.imu import vision_only

    prod, _ = _pair(True)
    src = SyntheticStereoSource(seed=5, n_frames=4)
    smp = _samples(src, 3)
    prod.begin(smp[0][2])
    s = prod.step(prod.st, *smp[1])
    rng = np.random.default_rng(11)
    for trial in range(20):
        A = rng.standard_normal((6, 6))
        cov = (A @ A.T + 6 * np.eye(6)) * 1e-10   # the vision well determined: H_v positive definite
        T = np.eye(4)
        T[:3, :3] = Rotation.from_rotvec(rng.normal(0, 0.01, 3)).as_matrix() @ s.R_rel
        T[:3, 3] = s.t_rel + rng.normal(0, 1e-3, 3)
        sigma2 = float(rng.uniform(0.5, 2.0))
        got_T, got_C = vision_only(T, cov, sigma2, s)
        want_T, want_C = OI.vision_only(T, cov, sigma2, (s.R_rel, s.w_rot, s.t_rel, s.w_trans))
        np.testing.assert_allclose(got_T, want_T, rtol=0, atol=1e-12)
        np.testing.assert_allclose(got_C, want_C, rtol=1e-9, atol=1e-22)
        if trial == 0:
            assert np.abs(got_T - T).max() > 0   # the prior acted: the vision-only pose differs
    # pass-through: no sigma^2, no prior weight, and a vision normal matrix that is not positive definite
    cov = np.eye(6) * 1e-6
    for sig, st in ((0.0, s), (1.0, type(s)(s.dt, s.gyro, s.w, s.R_rel, s.t_rel, 0.0, 0.0, s.v1, s.var_v1))):
        got_T, got_C = vision_only(T, cov, sig, st)
        np.testing.assert_array_equal(got_T, T)
        np.testing.assert_array_equal(got_C, cov)
    big = type(s)(s.dt, s.gyro, s.w, s.R_rel, s.t_rel, 1e12, 1e12, s.v1, s.var_v1)
    got_T, got_C = vision_only(T, cov, 1.0, big)
    np.testing.assert_array_equal(got_T, T)


def test_preintegration_matches_oracle():
    """tslam_imu_preintegrate (the product's inertial factor record) against the spec
    oracle/numpy_ba.py preintegrate on the synthetic IMU, with biases and w_prev, to 1e-12."""
    from oracle.numpy_ba import preintegrate

    src = SyntheticStereoSource(seed=0, imu=True, n_frames=60, gyro_bias=np.array([0.01, -0.02, 0.005]))
    ri = _rect_R_imu(src)
    noise = ImuNoise()
    prod = ImuPropagator(ri, noise, lever=LEVER)
    dt = 1.0 / src.fps
    bg, ba = np.array([0.004, -0.01, 0.002]), np.array([0.03, 0.01, -0.02])
    for i0, wp in ((5, None), (12, np.array([0.1, -0.2, 0.05]))):
        smp = [(dt, src.imu_sample(k)["gyroscope"], src.imu_sample(k)["accelerometer"]) for k in range(i0 + 1, i0 + 6)]
        got = prod.preintegrate(smp, bg, ba, wp)
        want = preintegrate(smp, ri, bg, ba, LEVER, w_prev=wp, acc_density=noise.acc_density,
                            gyro_density=noise.gyro_density, r_floor=1e-3, acc_rw=noise.acc_random_walk,
                            gyro_rw=noise.gyro_random_walk, ba_floor=1e-3, bg_floor=1e-3)
        assert got.size == want.size == 80 and got[30] > 0 and got[31] > 0 and got[71] > 0
        np.testing.assert_allclose(got, want, rtol=1e-12, atol=1e-14)
    prod.begin(src.imu_sample(0)["accelerometer"])
    g = prod.gravity()
    assert abs(np.linalg.norm(g) - 9.81) < 1e-12
