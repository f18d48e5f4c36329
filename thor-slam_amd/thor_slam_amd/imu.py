"""Visual-inertial motion priors: gyroscope + accelerometer.

The reference runs cuVSLAM with ``enable_imu_fusion:=true`` (``Makefile:81``) on the OAK's IMU
(one ``IMUData`` per synchronised frame set, ``thor_slam/camera/types.py:268-269``,
``rig.py:403-407``) with the noise model of ``launch/thor_visual_slam.launch.py:82-93``.  Here
the host keeps a small inertial state — camera orientation, world velocity, world gravity, the
accelerometer and gyroscope biases and their variances — and turns every frame's IMU sample into a
motion prior that the device's Gauss-Newton uses (``tslam_set_motion_prior``): the bias-corrected
gyro rotation with a weight from the gyroscope noise density and the bias uncertainty, and the
translation predicted from velocity, gravity and the specific force (less the IMU lever arm's
centripetal and tangential terms) with its weight.  A frame the vision loses but the prior covers
is chained with the prediction on the device, so the trajectory runs through visual dropouts.
After every batch the state absorbs the tracked motions (velocity, accelerometer-bias and
gyroscope-bias corrections weighted by the visual covariance).

Frames: the rectified-left camera of pair 0; the filter's world is that camera where the filter
started.  T_rel maps frame-k points to frame k+1 (X' = R_rel X + t_rel).  The spec, with the
operation order the checker follows, is ``oracle/numpy_imu.py`` (not imported here).
"""

from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np
from scipy.spatial.transform import Rotation

GRAVITY = 9.81


@dataclass
class ImuNoise:
    """Noise model (launch/thor_visual_slam.launch.py:82-93 densities) and the filter's priors."""
    gyro_density: float = 8.27e-5          # rad/s/sqrt(Hz)
    gyro_random_walk: float = 1e-8         # rad/s^2/sqrt(Hz)
    acc_density: float = 2.553e-3          # m/s^2/sqrt(Hz)
    acc_random_walk: float = 1.0493e-4     # m/s^3/sqrt(Hz)
    rot_floor: float = 2e-4                # rad, added in quadrature to the predicted rotation's std
    trans_floor: float = 1e-3              # m, added in quadrature to the predicted translation's std
    v0_sigma: float = 1.0                  # m/s, initial velocity std
    ba0_sigma: float = 0.05                # m/s^2, initial accelerometer-bias std
    bg0_sigma: float = 0.01                # rad/s, initial gyroscope-bias std
    vis_rot_floor: float = 1e-4            # rad, the vision's per-frame rotation error beyond its covariance


@dataclass
class InertialState:
    R: np.ndarray = field(default_factory=lambda: np.eye(3))    # world_R_cam
    v: np.ndarray = field(default_factory=lambda: np.zeros(3))  # world velocity [m/s]
    ba: np.ndarray = field(default_factory=lambda: np.zeros(3))  # accelerometer bias, IMU axes
    var_v: float = 1.0
    var_b: float = 0.0025
    bg: np.ndarray = field(default_factory=lambda: np.zeros(3))  # gyroscope bias, IMU axes
    var_g: float = 1e-4
    w_prev: np.ndarray | None = None                             # previous interval's camera-axes rate

    def copy(self) -> "InertialState":
        return InertialState(self.R.copy(), self.v.copy(), self.ba.copy(), self.var_v, self.var_b, self.bg.copy(),
                             self.var_g, None if self.w_prev is None else self.w_prev.copy())


@dataclass
class Step:
    """One frame interval's prediction."""
    dt: float
    gyro: np.ndarray
    w: np.ndarray           # bias-corrected rate, camera axes
    R_rel: np.ndarray
    t_rel: np.ndarray
    w_rot: float
    w_trans: float
    v1: np.ndarray | None
    var_v1: float


class ImuPropagator:
    """IMU priors for the device and the inertial state behind them.  ``accel=False`` is the
    gyro-only filter (rotation prior + gyroscope bias; no translation prior)."""

    def __init__(self, rect_R_imu: np.ndarray, noise: ImuNoise | None = None, lever: np.ndarray | None = None,
                 accel: bool = True):
        n = noise or ImuNoise()
        self.Ri = np.asarray(rect_R_imu, dtype=np.float64)
        self.na, self.rw = float(n.acc_density), float(n.acc_random_walk)
        self.ng, self.rwg = float(n.gyro_density), float(n.gyro_random_walk)
        self.rot_floor2, self.floor2 = float(n.rot_floor) ** 2, float(n.trans_floor) ** 2
        self.vis_floor = float(n.vis_rot_floor)
        self.v0_var, self.ba0_var, self.bg0_var = float(n.v0_sigma) ** 2, float(n.ba0_sigma) ** 2, float(n.bg0_sigma) ** 2
        self.r = np.zeros(3) if lever is None else np.asarray(lever, dtype=np.float64).reshape(3)
        self.accel = bool(accel)
        self.g: np.ndarray | None = None
        self.st = InertialState()
        self._ready = False

    @property
    def ready(self) -> bool:
        return self._ready

    def reset(self) -> None:
        self.g = None
        self.st = InertialState()
        self._ready = False

    def begin(self, accel: np.ndarray | None = None) -> None:
        """Start at rest: the specific force is gravity's reaction (gyro-only: no sample needed)."""
        self.g = np.zeros(3)
        if self.accel:
            f = self.Ri @ np.asarray(accel, dtype=np.float64)
            self.g = -GRAVITY * f / np.linalg.norm(f)
        self.st = InertialState(var_v=self.v0_var, var_b=self.ba0_var, var_g=self.bg0_var)
        self._ready = True

    def step(self, st: InertialState, dt: float, gyro: np.ndarray, accel: np.ndarray | None) -> Step:
        gyro = np.asarray(gyro, dtype=np.float64)
        w = self.Ri @ (gyro - st.bg)
        r_rel = Rotation.from_rotvec(-w * dt).as_matrix()
        w_rot = 1.0 / (self.ng ** 2 * dt + st.var_g * dt * dt + self.rot_floor2)
        if not self.accel:
            return Step(dt, gyro, w, r_rel, np.zeros(3), w_rot, 0.0, None, 0.0)
        alpha = np.zeros(3) if st.w_prev is None else (w - st.w_prev) / dt
        w_w, al_w, r_w = st.R @ w, st.R @ alpha, st.R @ self.r
        a_w = (st.R @ (self.Ri @ (np.asarray(accel, dtype=np.float64) - st.ba)) + self.g
               - np.cross(w_w, np.cross(w_w, r_w)) - np.cross(al_w, r_w))
        centre = st.R.T @ (st.v * dt + 0.5 * a_w * dt * dt)   # new camera centre, old camera axes
        var_t = st.var_v * dt ** 2 + self.na ** 2 * dt ** 3 / 3.0 + st.var_b * dt ** 4 / 4.0 + self.floor2
        return Step(dt, gyro, w, r_rel, -(r_rel @ centre), w_rot, 1.0 / var_t, st.v + a_w * dt,
                    st.var_v + self.na ** 2 * dt + st.var_b * dt * dt)

    def coast(self, st: InertialState, s: Step) -> InertialState:
        """No visual motion for the interval: the state follows the IMU."""
        if not self.accel:
            return InertialState(st.R @ s.R_rel.T, st.v, st.ba, st.var_v, st.var_b, st.bg,
                                 st.var_g + self.rwg ** 2 * s.dt, s.w)
        return InertialState(st.R @ s.R_rel.T, s.v1, st.ba, s.var_v1, st.var_b + self.rw ** 2 * s.dt, st.bg,
                             st.var_g + self.rwg ** 2 * s.dt, s.w)

    def correct(self, st: InertialState, s: Step, t_rel: np.ndarray, cov: np.ndarray) -> InertialState:
        """A tracked interval: gyroscope bias (and, with the accelerometer leg, velocity and
        accelerometer bias) pulled towards the visual motion."""
        dt = s.dt
        rv = t_rel[:3, :3]
        var_g1 = st.var_g + self.rwg ** 2 * dt
        w_v = -Rotation.from_matrix(rv).as_rotvec() / dt
        z = s.gyro - self.Ri.T @ w_v
        var_z = np.trace(cov[3:, 3:]) / 3.0 / dt ** 2 + self.ng ** 2 / dt + (self.vis_floor / dt) ** 2
        kg = var_g1 / (var_g1 + var_z)
        bg, var_g = st.bg + kg * (z - st.bg), (1.0 - kg) * var_g1
        if not self.accel:
            return InertialState(st.R @ rv.T, st.v, st.ba, st.var_v, st.var_b, bg, var_g, s.w)
        v_vis = (st.R @ (-(rv.T @ t_rel[:3, 3]))) / dt
        var_vis = np.trace(cov[:3, :3]) / 3.0 / dt ** 2
        innov = v_vis - s.v1
        k = s.var_v1 / (s.var_v1 + var_vis)
        var_b1 = st.var_b + self.rw ** 2 * dt
        kb = var_b1 / (var_b1 + (var_vis + s.var_v1) / dt ** 2 + self.na ** 2 / dt)
        e_imu = self.Ri.T @ (st.R.T @ (innov / dt))
        return InertialState(st.R @ rv.T, s.v1 + k * innov, st.ba - kb * e_imu, (1.0 - k) * s.var_v1,
                             (1.0 - kb) * var_b1, bg, var_g, s.w)

    def batch_priors(self, samples: list) -> list[Step | None]:
        """Per frame of the next batch (``samples`` = [(dt | None, gyro, accel)]): its prediction
        from the current state coasted over the batch's earlier frames."""
        st = self.st.copy()
        out: list[Step | None] = []
        for dt, gy, ac in samples:
            if dt is None or not self.ready:
                out.append(None)
                continue
            s = self.step(st, dt, gy, ac)
            out.append(s)
            st = self.coast(st, s)
        return out

    def absorb(self, samples: list, status: np.ndarray, t_rel: np.ndarray, cov: np.ndarray) -> None:
        """The batch's results in the filter's camera: status [n], T_rel [n][4][4], cov [n][6][6]."""
        for k, (dt, gy, ac) in enumerate(samples):
            if dt is None or not self.ready:
                continue
            s = self.step(self.st, dt, gy, ac)
            self.st = self.correct(self.st, s, t_rel[k], cov[k]) if int(status[k]) == 0 else self.coast(self.st, s)


def vision_only(T: np.ndarray, cov: np.ndarray, sigma2: float, step: Step) -> tuple[np.ndarray, np.ndarray]:
    """The vision-only motion and covariance behind a solution the device weighted with ``step``'s
    prior: one Gauss-Newton step on the vision alone from the solution, with the vision's normal
    matrix H_v = sigma^2 C^-1 - diag(W_t I, W_r I) in (rho, omega) and A7's left Cayley update.
    The gyroscope-bias update needs it: a rotation the gyro prior already pulled cannot show the
    bias.  (T, cov) unchanged when no prior acted or H_v is not positive definite."""
    if not sigma2 > 0.0 or not (step.w_rot > 0.0 or step.w_trans > 0.0):
        return T, cov
    h = sigma2 * np.linalg.inv(cov)
    hv = h.copy()
    hv[:3, :3] -= step.w_trans * np.eye(3)
    hv[3:, 3:] -= step.w_rot * np.eye(3)
    hv = 0.5 * (hv + hv.T)
    try:
        np.linalg.cholesky(hv)
    except np.linalg.LinAlgError:
        return T, cov
    R, t = T[:3, :3], T[:3, 3]
    a = step.R_rel @ R.T
    delta = 0.5 * np.array([a[2, 1] - a[1, 2], a[0, 2] - a[2, 0], a[1, 0] - a[0, 1]])
    d = np.linalg.solve(hv, np.concatenate([step.w_trans * (t - step.t_rel), -step.w_rot * delta]))
    w0, w1, w2 = d[3:]
    A = np.array([[0.0, -w2, w1], [w2, 0.0, -w0], [-w1, w0, 0.0]])
    ru = np.eye(3) + (4.0 / (4.0 + (w0 * w0 + w1 * w1) + w2 * w2)) * (A + 0.5 * (A @ A))
    out = np.eye(4)
    out[:3, :3] = ru @ R
    out[:3, 3] = ru @ t + d[:3]
    return out, sigma2 * np.linalg.inv(hv)
