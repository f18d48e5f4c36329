"""Visual-inertial motion priors: gyroscope + accelerometer.

The reference runs cuVSLAM with ``enable_imu_fusion:=true`` (``Makefile:81``) on the OAK's IMU
(one ``IMUData`` per synchronised frame set, ``thor_slam/camera/types.py:268-269``,
``rig.py:403-407``) with the noise model of ``launch/thor_visual_slam.launch.py:82-93``.  Here
the host keeps a small inertial state — camera orientation, world velocity, world gravity and the
accelerometer bias — and turns every frame's IMU sample into a motion prior that the device's
Gauss-Newton uses (``tslam_set_motion_prior``): the gyro's relative rotation and the translation
predicted from velocity, gravity and specific force, each with its weight.  A frame the vision
loses but the prior covers is chained with the prediction on the device, so the trajectory runs
through visual dropouts.  After every batch the state absorbs the tracked motions (velocity and
bias corrections weighted by the visual covariance).

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
class InertialState:
    R: np.ndarray = field(default_factory=lambda: np.eye(3))    # world_R_cam
    v: np.ndarray = field(default_factory=lambda: np.zeros(3))  # world velocity [m/s]
    ba: np.ndarray = field(default_factory=lambda: np.zeros(3))  # accelerometer bias, IMU axes
    var_v: float = 1.0
    var_b: float = 0.0025

    def copy(self) -> "InertialState":
        return InertialState(self.R.copy(), self.v.copy(), self.ba.copy(), self.var_v, self.var_b)


@dataclass
class Step:
    """One frame interval's prediction."""
    dt: float
    R_rel: np.ndarray
    t_rel: np.ndarray
    w_rot: float
    w_trans: float
    v1: np.ndarray
    var_v1: float


class ImuPropagator:
    """Gyro + accelerometer priors for the device and the inertial state behind them."""

    def __init__(self, rect_R_imu: np.ndarray, acc_density: float, acc_random_walk: float, rot_sigma: float,
                 trans_floor: float, v0_sigma: float = 1.0, ba0_sigma: float = 0.05):
        self.Ri = np.asarray(rect_R_imu, dtype=np.float64)
        self.na2 = float(acc_density) ** 2
        self.rw2 = float(acc_random_walk) ** 2
        self.w_rot = 1.0 / float(rot_sigma) ** 2
        self.floor2 = float(trans_floor) ** 2
        self.v0_var, self.ba0_var = float(v0_sigma) ** 2, float(ba0_sigma) ** 2
        self.g: np.ndarray | None = None
        self.st = InertialState()

    @property
    def ready(self) -> bool:
        return self.g is not None

    def reset(self) -> None:
        self.g = None
        self.st = InertialState()

    def begin(self, accel: np.ndarray) -> None:
        """Start at rest: the specific force is gravity's reaction."""
        f = self.Ri @ np.asarray(accel, dtype=np.float64)
        self.g = -GRAVITY * f / np.linalg.norm(f)
        self.st = InertialState(var_v=self.v0_var, var_b=self.ba0_var)

    def step(self, st: InertialState, dt: float, gyro: np.ndarray, accel: np.ndarray) -> Step:
        w = self.Ri @ np.asarray(gyro, dtype=np.float64)
        r_rel = Rotation.from_rotvec(-w * dt).as_matrix()
        a_w = st.R @ (self.Ri @ (np.asarray(accel, dtype=np.float64) - st.ba)) + self.g
        centre = st.R.T @ (st.v * dt + 0.5 * a_w * dt * dt)   # new camera centre, old camera axes
        var_t = st.var_v * dt ** 2 + self.na2 * dt ** 3 / 3.0 + st.var_b * dt ** 4 / 4.0 + self.floor2
        return Step(dt, r_rel, -(r_rel @ centre), self.w_rot, 1.0 / var_t, st.v + a_w * dt,
                    st.var_v + self.na2 * dt + st.var_b * dt * dt)

    def coast(self, st: InertialState, s: Step) -> InertialState:
        """No visual motion for the interval: the state follows the IMU."""
        return InertialState(st.R @ s.R_rel.T, s.v1, st.ba, s.var_v1, st.var_b + self.rw2 * s.dt)

    def correct(self, st: InertialState, s: Step, t_rel: np.ndarray, cov: np.ndarray) -> InertialState:
        """A tracked interval: velocity and bias pulled towards the visual motion."""
        dt = s.dt
        rv = t_rel[:3, :3]
        v_vis = (st.R @ (-(rv.T @ t_rel[:3, 3]))) / dt
        var_vis = np.trace(cov[:3, :3]) / 3.0 / dt ** 2
        innov = v_vis - s.v1
        k = s.var_v1 / (s.var_v1 + var_vis)
        var_b1 = st.var_b + self.rw2 * dt
        kb = var_b1 / (var_b1 + (var_vis + s.var_v1) / dt ** 2 + self.na2 / dt)
        e_imu = self.Ri.T @ (st.R.T @ (innov / dt))
        return InertialState(st.R @ rv.T, s.v1 + k * innov, st.ba - kb * e_imu, (1.0 - k) * s.var_v1,
                             (1.0 - kb) * var_b1)

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
        """The batch's results (pair 0): status [n], T_rel [n][4][4], cov [n][6][6]."""
        for k, (dt, gy, ac) in enumerate(samples):
            if dt is None or not self.ready:
                continue
            s = self.step(self.st, dt, gy, ac)
            self.st = self.correct(self.st, s, t_rel[k], cov[k]) if int(status[k]) == 0 else self.coast(self.st, s)
