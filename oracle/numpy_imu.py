"""SURVEY.md §8f item 2 — the accelerometer leg of IMU fusion, CPU restatement.

TEST INFRASTRUCTURE (see ``oracle/__init__.py``): the checker for the product's IMU filter
(``thor_slam_amd/imu.py``) and, through ``run_sequence``, for the device's motion-prior terms
(``k_refine``) and IMU chaining (``k_chain``).  cuVSLAM's visual-inertial fusion is closed
(SURVEY.md §8c), so this file is the spec; parity against the reference is unpinned like rows
A2-A8.  The reference supplies the inputs and the noise model: one IMU sample per synchronised
frame set (``SynchronizedFrameSet.sensor_data``, ``thor_slam/camera/types.py:268-269``, filled by
``rig.py:403-407`` from the OAK's ``IMUData``, ``luxonis.py:21-35``) and the densities of
``launch/thor_visual_slam.launch.py:82-93`` (accelerometer 2.553e-3 m/s^2/sqrt(Hz), random walk
1.0493e-4 m/s^3/sqrt(Hz)).

Spec.  Frames are the rectified-left camera of pair 0; the world is that camera at the first
frame (the frame ``T_abs`` is expressed in).  T_rel maps frame-k points to frame k+1:
X_{k+1} = R_rel X_k + t_rel; the camera pose advances as R <- R R_rel^T, p <- p + R c with the
new camera centre c = -R_rel^T t_rel.  State after frame k: R, v (world velocity), g (world
gravity), b_a (accelerometer bias, IMU axes), var_v, var_b (isotropic variances).

* start (first frame, INIT): R = I, v = 0, var_v = v0_sigma^2, b_a = 0, var_b = ba0_sigma^2,
  g = -9.81 f / |f| with f = rect_R_imu a_0 (the specific force at rest is -g);
* predict (sample of frame k+1: dt, gyro w, accel a):
    R_rel = exp(-[rect_R_imu w dt]x)                    (the gyro rotation prior, as before)
    a_w = R rect_R_imu (a - b_a) + g,  dp = v dt + a_w dt^2 / 2,  c = R^T dp,  t_rel = -R_rel c
    v' = v + a_w dt,  var_v' = var_v + n_a^2 dt + var_b dt^2
    var_t = var_v dt^2 + n_a^2 dt^3 / 3 + var_b dt^4 / 4 + floor^2,  W_t = 1 / var_t,
    W_r = 1 / rot_sigma^2
  (weights in the solver's units: 1 px of reprojection error = 1 unit, as the rotation prior);
* update with frame k+1's result:
    tracked (status 0, visual T_rel = [R_v | t_v], 6x6 covariance C): R <- R R_v^T;
      v_vis = R c_v / dt (c_v = -R_v^T t_v, R before the update), var_vis = tr(C[:3,:3]) / 3 / dt^2;
      K = var_v' / (var_v' + var_vis), v <- v' + K (v_vis - v'), var_v <- (1 - K) var_v';
      e = rect_R_imu^T R^T (v_vis - v') / dt, var_b' = var_b + rw_a^2 dt,
      K_b = var_b' / (var_b' + (var_vis + var_v') / dt^2 + n_a^2 / dt), b_a <- b_a - K_b e, var_b <- (1 - K_b) var_b'
    not tracked: R <- R R_rel^T, v <- v', var_v <- var_v', var_b <- var_b + rw_a^2 dt;
* a batch of frames gets its priors from the state at the batch start propagated by
  IMU-only steps (the device solves a batch's frames in parallel); after the batch the filter
  runs predict + update frame by frame on the results;
* the device: W_t adds W_t I to the translation block of A7's Gauss-Newton and W_t (t_rel - t) to
  its gradient (``numpy_slam.refine``); an untracked frame with W_t > 0 is chained with the
  predicted [R_rel | t_rel] (``OracleTracker._advance``).
"""

from __future__ import annotations

import numpy as np
from scipy.spatial.transform import Rotation

GRAVITY = 9.81


class ImuFilter:
    def __init__(self, rect_R_imu: np.ndarray, acc_density: float = 2.553e-3, acc_random_walk: float = 1.0493e-4,
                 rot_sigma: float = 2e-3, trans_floor: float = 1e-3, v0_sigma: float = 1.0, ba0_sigma: float = 0.05):
        self.Ri = np.asarray(rect_R_imu, dtype=np.float64)
        self.na, self.rw = float(acc_density), float(acc_random_walk)
        self.rot_sigma, self.floor = float(rot_sigma), float(trans_floor)
        self.v0_sigma, self.ba0_sigma = float(v0_sigma), float(ba0_sigma)
        self.ready = False

    def start(self, accel: np.ndarray) -> None:
        f = self.Ri @ np.asarray(accel, dtype=np.float64)
        self.R = np.eye(3)
        self.v = np.zeros(3)
        self.g = -GRAVITY * f / np.linalg.norm(f)
        self.ba = np.zeros(3)
        self.var_v = self.v0_sigma ** 2
        self.var_b = self.ba0_sigma ** 2
        self.ready = True

    def state(self) -> tuple:
        return (self.R.copy(), self.v.copy(), self.ba.copy(), self.var_v, self.var_b)

    def set_state(self, st: tuple) -> None:
        self.R, self.v, self.ba, self.var_v, self.var_b = st[0].copy(), st[1].copy(), st[2].copy(), st[3], st[4]

    def predict(self, dt: float, gyro: np.ndarray, accel: np.ndarray) -> dict:
        w = self.Ri @ np.asarray(gyro, dtype=np.float64)
        r_rel = Rotation.from_rotvec(-w * dt).as_matrix()
        a_w = self.R @ (self.Ri @ (np.asarray(accel, dtype=np.float64) - self.ba)) + self.g
        dp = self.v * dt + 0.5 * a_w * dt * dt
        c = self.R.T @ dp
        var_t = self.var_v * dt ** 2 + self.na ** 2 * dt ** 3 / 3.0 + self.var_b * dt ** 4 / 4.0 + self.floor ** 2
        return {"dt": dt, "R_rel": r_rel, "t_rel": -(r_rel @ c), "W_r": 1.0 / self.rot_sigma ** 2, "W_t": 1.0 / var_t,
                "v1": self.v + a_w * dt, "var_v1": self.var_v + self.na ** 2 * dt + self.var_b * dt * dt}

    def update(self, pred: dict, status: int, t_rel: np.ndarray | None = None, cov: np.ndarray | None = None) -> None:
        dt = pred["dt"]
        var_b1 = self.var_b + self.rw ** 2 * dt
        if status == 0:
            rv, tv = t_rel[:3, :3], t_rel[:3, 3]
            d_w = self.R @ (-(rv.T @ tv))
            v_vis = d_w / dt
            var_vis = np.trace(cov[:3, :3]) / 3.0 / dt ** 2
            k = pred["var_v1"] / (pred["var_v1"] + var_vis)
            e = self.Ri.T @ (self.R.T @ ((v_vis - pred["v1"]) / dt))
            kb = var_b1 / (var_b1 + (var_vis + pred["var_v1"]) / dt ** 2 + self.na ** 2 / dt)
            self.v = pred["v1"] + k * (v_vis - pred["v1"])
            self.var_v = (1.0 - k) * pred["var_v1"]
            self.ba = self.ba - kb * e
            self.var_b = (1.0 - kb) * var_b1
            self.R = self.R @ rv.T
        else:
            self.R = self.R @ pred["R_rel"].T
            self.v = pred["v1"]
            self.var_v = pred["var_v1"]
            self.var_b = var_b1


def batch_priors(filt: ImuFilter, samples: list) -> list:
    """Priors (R_rel, W_r, t_rel, W_t) of a batch's frames from the filter's current state,
    propagated by IMU-only steps; ``samples`` = [(dt, gyro, accel)] (dt None: no prior)."""
    saved = filt.state()
    out = []
    for dt, gy, ac in samples:
        if dt is None or not filt.ready:
            out.append(None)
            continue
        p = filt.predict(dt, gy, ac)
        out.append((p["R_rel"], p["W_r"], p["t_rel"], p["W_t"]))
        filt.update(p, 1)
    filt.set_state(saved)
    return out


def run_sequence(tracker, frames: np.ndarray, samples: list, batch: int, filt: ImuFilter | None) -> list:
    """The engine's batch flow on the oracle tracker: ``samples[i]`` = (dt, gyro, accel) of frame
    i (dt None for the first).  Returns the tracker's per-frame results."""
    results = []
    for b0 in range(0, len(frames), batch):
        idx = range(b0, min(b0 + batch, len(frames)))
        if filt is not None and not filt.ready:
            filt.start(samples[b0][2])
        priors = batch_priors(filt, [samples[i] for i in idx]) if filt is not None else [None] * len(idx)
        res = [tracker.step(frames[i, 0], frames[i, 1], prior=pr) for i, pr in zip(idx, priors)]
        if filt is not None:
            for i, r in zip(idx, res):
                dt, gy, ac = samples[i]
                if dt is None:
                    continue
                filt.update(filt.predict(dt, gy, ac), int(r["status"]), r["T"], r["cov"])
        results += res
    return results
