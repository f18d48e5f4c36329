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
started.  T_rel maps frame-k points to frame k+1 (X' = R_rel X + t_rel).  The filter itself is
native (``csrc/tslam_imu.cpp``, C-ABI ``tslam_imu_*`` in ``include/tslam.h``); this module binds
it and keeps the state / step records as dataclasses.  The spec, with the operation order the
checker follows, is ``oracle/numpy_imu.py`` (not imported here).
"""

from __future__ import annotations

from dataclasses import dataclass, field

import ctypes

import numpy as np

from . import _lib

GRAVITY = 9.81   # m/s^2 (csrc/tslam_imu.cpp)


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


def _c_state(st: InertialState) -> _lib.ImuState:
    c = _lib.ImuState()
    c.R[:] = [float(x) for x in np.asarray(st.R, dtype=np.float64).reshape(9)]
    c.v[:] = [float(x) for x in np.asarray(st.v, dtype=np.float64)]
    c.ba[:] = [float(x) for x in np.asarray(st.ba, dtype=np.float64)]
    c.bg[:] = [float(x) for x in np.asarray(st.bg, dtype=np.float64)]
    c.var_v, c.var_b, c.var_g = float(st.var_v), float(st.var_b), float(st.var_g)
    if st.w_prev is not None:
        c.w_prev[:] = [float(x) for x in np.asarray(st.w_prev, dtype=np.float64)]
        c.has_w_prev = 1
    return c


def _py_state(c: _lib.ImuState) -> InertialState:
    return InertialState(np.array(c.R[:]).reshape(3, 3), np.array(c.v[:]), np.array(c.ba[:]), c.var_v, c.var_b,
                         np.array(c.bg[:]), c.var_g, np.array(c.w_prev[:]) if c.has_w_prev else None)


def _c_step(s: Step) -> _lib.ImuStep:
    c = _lib.ImuStep()
    c.dt = float(s.dt)
    c.gyro[:] = [float(x) for x in np.asarray(s.gyro, dtype=np.float64)]
    c.w[:] = [float(x) for x in np.asarray(s.w, dtype=np.float64)]
    c.R_rel[:] = [float(x) for x in np.asarray(s.R_rel, dtype=np.float64).reshape(9)]
    c.t_rel[:] = [float(x) for x in np.asarray(s.t_rel, dtype=np.float64)]
    c.w_rot, c.w_trans, c.var_v1 = float(s.w_rot), float(s.w_trans), float(s.var_v1)
    if s.v1 is not None:
        c.v1[:] = [float(x) for x in np.asarray(s.v1, dtype=np.float64)]
        c.has_v1 = 1
    return c


def _py_step(c: _lib.ImuStep) -> Step:
    return Step(c.dt, np.array(c.gyro[:]), np.array(c.w[:]), np.array(c.R_rel[:]).reshape(3, 3), np.array(c.t_rel[:]),
                c.w_rot, c.w_trans, np.array(c.v1[:]) if c.has_v1 else None, c.var_v1)


def _vec(x) -> ctypes.Array:
    return (ctypes.c_double * 3)(*[float(v) for v in np.asarray(x, dtype=np.float64).reshape(3)])


class ImuPropagator:
    """IMU priors for the device and the inertial state behind them, on the native filter
    (``tslam_imu_*``).  ``accel=False`` is the gyro-only filter (rotation prior + gyroscope bias;
    no translation prior)."""

    def __init__(self, rect_R_imu: np.ndarray, noise: ImuNoise | None = None, lever: np.ndarray | None = None,
                 accel: bool = True):
        n = noise or ImuNoise()
        self.lib = _lib.load_library()
        ri = (ctypes.c_double * 9)(*[float(v) for v in np.asarray(rect_R_imu, dtype=np.float64).reshape(9)])
        nz = (ctypes.c_double * 10)(n.gyro_density, n.gyro_random_walk, n.acc_density, n.acc_random_walk, n.rot_floor,
                                    n.trans_floor, n.v0_sigma, n.ba0_sigma, n.bg0_sigma, n.vis_rot_floor)
        lv = _vec(np.zeros(3) if lever is None else lever)
        self.accel = bool(accel)
        self._f = ctypes.c_void_p()
        _lib._check(self.lib.tslam_imu_create(ri, nz, lv, int(self.accel), ctypes.byref(self._f)))

    def __del__(self):
        f = getattr(self, "_f", None)
        if f:
            self.lib.tslam_imu_destroy(f)
            self._f = None

    @property
    def ready(self) -> bool:
        return bool(self.lib.tslam_imu_ready(self._f))

    @property
    def st(self) -> InertialState:
        c = _lib.ImuState()
        _lib._check(self.lib.tslam_imu_get_state(self._f, ctypes.byref(c)))
        return _py_state(c)

    @st.setter
    def st(self, value: InertialState) -> None:
        c = _c_state(value)
        _lib._check(self.lib.tslam_imu_set_state(self._f, ctypes.byref(c)))

    def reset(self) -> None:
        _lib._check(self.lib.tslam_imu_reset(self._f))

    def begin(self, accel: np.ndarray | None = None) -> None:
        """Start at rest: the specific force is gravity's reaction (gyro-only: no sample needed)."""
        _lib._check(self.lib.tslam_imu_begin(self._f, _vec(accel) if (self.accel and accel is not None) else None))

    def step(self, st: InertialState, dt: float, gyro: np.ndarray, accel: np.ndarray | None) -> Step:
        c, out = _c_state(st), _lib.ImuStep()
        _lib._check(self.lib.tslam_imu_predict(self._f, ctypes.byref(c), float(dt), _vec(gyro),
                                               _vec(accel) if accel is not None else None, ctypes.byref(out)))
        return _py_step(out)

    def coast(self, st: InertialState, s: Step) -> InertialState:
        """No visual motion for the interval: the state follows the IMU."""
        c, cs, out = _c_state(st), _c_step(s), _lib.ImuState()
        _lib._check(self.lib.tslam_imu_coast(self._f, ctypes.byref(c), ctypes.byref(cs), ctypes.byref(out)))
        return _py_state(out)

    def correct(self, st: InertialState, s: Step, t_rel: np.ndarray, cov: np.ndarray) -> InertialState:
        """A tracked interval: gyroscope bias (and, with the accelerometer leg, velocity and
        accelerometer bias) pulled towards the visual motion."""
        c, cs, out = _c_state(st), _c_step(s), _lib.ImuState()
        t = np.ascontiguousarray(t_rel, dtype=np.float64).reshape(16)
        cv = np.ascontiguousarray(cov, dtype=np.float64).reshape(36)
        _lib._check(self.lib.tslam_imu_correct(self._f, ctypes.byref(c), ctypes.byref(cs), t.ctypes.data, cv.ctypes.data,
                                               ctypes.byref(out)))
        return _py_state(out)

    def _arrays(self, samples: list):
        n = len(samples)
        dt = np.full(n, np.nan)
        gy = np.zeros((n, 3))
        ac = np.zeros((n, 3)) if self.accel else None
        for k, (d, g, a) in enumerate(samples):
            if d is None:
                continue
            dt[k] = float(d)
            gy[k] = np.asarray(g, dtype=np.float64)
            if ac is not None:
                ac[k] = np.asarray(a, dtype=np.float64) if a is not None else np.nan
        return n, dt, gy, ac

    def batch_priors(self, samples: list) -> list[Step | None]:
        """Per frame of the next batch (``samples`` = [(dt | None, gyro, accel)]): its prediction
        from the current state coasted over the batch's earlier frames (tslam_imu_batch_priors)."""
        n, dt, gy, ac = self._arrays(samples)
        out = (_lib.ImuStep * max(n, 1))()
        valid = np.zeros(max(n, 1), dtype=np.int32)
        _lib._check(self.lib.tslam_imu_batch_priors(self._f, n, dt.ctypes.data, gy.ctypes.data,
                                                    None if ac is None else ac.ctypes.data, out, valid.ctypes.data))
        return [_py_step(out[k]) if valid[k] else None for k in range(n)]

    def gravity(self) -> np.ndarray:
        """World gravity of the accelerometer filter (its camera-0 world; zeros before ``begin``)."""
        g = np.zeros(3)
        _lib._check(self.lib.tslam_imu_gravity(self._f, g.ctypes.data))
        return g

    def preintegrate(self, samples: list, bg: np.ndarray, ba: np.ndarray, w_prev: np.ndarray | None = None,
                     v_floor: float = 1e-2, p_floor: float = 1e-3, frame_R_imu: np.ndarray | None = None,
                     lever: np.ndarray | None = None, r_floor: float = 1e-3, ba_floor: float = 1e-3,
                     bg_floor: float = 1e-3) -> np.ndarray:
        """The local BA's inertial factor record (INE_RECORD doubles, tslam_ba_inertial_factor) of
        the frame intervals ``samples`` = [(dt, gyro, accel)] between two keyframes, in the filter's
        camera or (``frame_R_imu``, ``lever``) another rigid frame (tslam_imu_preintegrate)."""
        n = len(samples)
        dt = np.ascontiguousarray([float(d) for d, _, _ in samples], dtype=np.float64)
        gy = np.ascontiguousarray([np.asarray(g, dtype=np.float64).reshape(3) for _, g, _ in samples])
        ac = np.ascontiguousarray([np.asarray(a, dtype=np.float64).reshape(3) for _, _, a in samples])
        bgv = np.ascontiguousarray(bg, dtype=np.float64).reshape(3)
        bav = np.ascontiguousarray(ba, dtype=np.float64).reshape(3)
        wp = None if w_prev is None else np.ascontiguousarray(w_prev, dtype=np.float64).reshape(3)
        fr = None if frame_R_imu is None else np.ascontiguousarray(frame_R_imu, dtype=np.float64).reshape(9)
        lv = None if lever is None else np.ascontiguousarray(lever, dtype=np.float64).reshape(3)
        out = np.zeros(_lib.INE_RECORD)
        _lib._check(self.lib.tslam_imu_preintegrate(self._f, n, dt.ctypes.data, gy.ctypes.data, ac.ctypes.data,
                                                    bgv.ctypes.data, bav.ctypes.data, None if wp is None else wp.ctypes.data,
                                                    None if fr is None else fr.ctypes.data,
                                                    None if lv is None else lv.ctypes.data,
                                                    float(v_floor), float(p_floor), float(r_floor), float(ba_floor),
                                                    float(bg_floor), out.ctypes.data))
        return out

    def absorb(self, samples: list, status: np.ndarray, t_rel: np.ndarray, cov: np.ndarray) -> None:
        """The batch's results in the filter's camera: status [n], T_rel [n][4][4], cov [n][6][6]
        (tslam_imu_absorb)."""
        n, dt, gy, ac = self._arrays(samples)
        st = np.ascontiguousarray(np.asarray(status)[:n], dtype=np.int32)
        t = np.ascontiguousarray(np.asarray(t_rel, dtype=np.float64)[:n].reshape(n, 16))
        cv = np.ascontiguousarray(np.asarray(cov, dtype=np.float64)[:n].reshape(n, 36))
        _lib._check(self.lib.tslam_imu_absorb(self._f, n, dt.ctypes.data, gy.ctypes.data,
                                              None if ac is None else ac.ctypes.data, st.ctypes.data, t.ctypes.data,
                                              cv.ctypes.data))


def vision_only(T: np.ndarray, cov: np.ndarray, sigma2: float, step: Step) -> tuple[np.ndarray, np.ndarray]:
    """The vision-only motion and covariance behind a solution the device weighted with ``step``'s
    prior: one Gauss-Newton step on the vision alone from the solution, with the vision's normal
    matrix H_v = sigma^2 C^-1 - diag(W_t I, W_r I) in (rho, omega) and A7's left Cayley update
    (tslam_imu_vision_only).  The gyroscope-bias update needs it: a rotation the gyro prior already
    pulled cannot show the bias.  (T, cov) unchanged when no prior acted or H_v is not positive
    definite."""
    lib = _lib.load_library()
    t = np.ascontiguousarray(T, dtype=np.float64).reshape(16)
    c = np.ascontiguousarray(cov, dtype=np.float64).reshape(36)
    t_out, c_out = np.zeros(16), np.zeros(36)
    cs = _c_step(step)
    _lib._check(lib.tslam_imu_vision_only(t.ctypes.data, c.ctypes.data, float(sigma2), ctypes.byref(cs),
                                          t_out.ctypes.data, c_out.ctypes.data))
    return t_out.reshape(4, 4), c_out.reshape(6, 6)
