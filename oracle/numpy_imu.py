"""SURVEY.md §8f item 2 — IMU fusion (gyroscope + accelerometer), CPU restatement.

TEST INFRASTRUCTURE (see ``oracle/__init__.py``): the checker for the product's IMU filter
(``thor_slam_amd/imu.py``) and, through ``run_sequence`` / ``run_rig_sequence``, for the device's
motion-prior terms (``k_refine``), IMU chaining (``k_chain``) and the rig's body-frame prediction
(``k_rig_prior``).  cuVSLAM's visual-inertial fusion is closed, so this file is the
spec; parity against the reference is unpinned like rows A2-A8.  The reference supplies the inputs
and the noise model: one IMU sample per synchronised frame set
(``SynchronizedFrameSet.sensor_data``, ``thor_slam/camera/types.py:268-269``, filled by
``rig.py:403-407`` from the OAK's ``IMUData``, ``luxonis.py:21-35``) and the four densities of
``launch/thor_visual_slam.launch.py:82-93``: gyroscope noise 8.27e-5 rad/s/sqrt(Hz), gyroscope
random walk 1e-8 rad/s^2/sqrt(Hz), accelerometer noise 2.553e-3 m/s^2/sqrt(Hz), accelerometer
random walk 1.0493e-4 m/s^3/sqrt(Hz).

Spec.  Frames are the rectified-left camera of pair 0; the world is that camera at the first
frame (the frame ``T_abs`` is expressed in).  T_rel maps frame-k points to frame k+1:
X_{k+1} = R_rel X_k + t_rel; the camera pose advances as R <- R R_rel^T, p <- p + R c with the
new camera centre c = -R_rel^T t_rel.  Ri = rect_R_imu (IMU axes -> camera axes), r = the IMU's
position in the camera frame (the lever arm).  State after frame k: R, v (world velocity), g
(world gravity), b_a (accelerometer bias, IMU axes), b_g (gyroscope bias, IMU axes), the
isotropic variances var_v, var_b, var_g, and w_prev (the previous interval's camera-axes rate).
vis_floor is the per-frame rotation error of the vision beyond its covariance (its errors are
correlated from frame to frame: measured ~1e-4 rad per frame on the synthetic sequences), so a
gyroscope bias is learnt from many frames, not from one.

* start: R = I, v = 0, b_a = b_g = 0, var_v = v0_sigma^2, var_b = ba0_sigma^2, var_g =
  bg0_sigma^2, w_prev = none; with the accelerometer leg g = -9.81 f / |f|, f = Ri a_0 (the specific
  force at rest is -g); a gyro-only filter needs no sample to start;
* predict (sample of frame k+1: dt, gyro w_m, accel a):
    w = Ri (w_m - b_g),  R_rel = exp(-[w dt]x),  W_r = 1 / (n_g^2 dt + var_g dt^2 + rot_floor^2)
  accelerometer leg (else t_rel = 0, W_t = 0):
    alpha = (w - w_prev) / dt (0 without w_prev);  w_w = R w, alpha_w = R alpha, r_w = R r
    a_w = R Ri (a - b_a) + g - w_w x (w_w x r_w) - alpha_w x r_w      (the camera's acceleration:
          the specific force at the IMU minus its centripetal and tangential lever-arm terms)
    dp = v dt + a_w dt^2 / 2,  c = R^T dp,  t_rel = -R_rel c
    v' = v + a_w dt,  var_v' = var_v + n_a^2 dt + var_b dt^2
    W_t = 1 / (var_v dt^2 + n_a^2 dt^3 / 3 + var_b dt^4 / 4 + trans_floor^2)
  (weights in the solver's units: 1 px of reprojection error = 1 unit);
* update with frame k+1's result (var_g' = var_g + rw_g^2 dt, var_b' = var_b + rw_a^2 dt):
    tracked (status 0, visual T_rel = [R_v | t_v], 6x6 covariance C in (rho, omega) order):
      gyro bias: w_v = -log(R_v) / dt (camera axes), z = w_m - Ri^T w_v,
        var_z = tr(C[3:,3:]) / 3 / dt^2 + n_g^2 / dt + (vis_floor / dt)^2, K_g = var_g' / (var_g' + var_z),
        b_g <- b_g + K_g (z - b_g), var_g <- (1 - K_g) var_g';
      accelerometer leg: v_vis = R c_v / dt (c_v = -R_v^T t_v, R before the update),
        var_vis = tr(C[:3,:3]) / 3 / dt^2, K = var_v' / (var_v' + var_vis),
        v <- v' + K (v_vis - v'), var_v <- (1 - K) var_v';
        e = Ri^T R^T (v_vis - v') / dt, K_b = var_b' / (var_b' + (var_vis + var_v') / dt^2 + n_a^2 / dt),
        b_a <- b_a - K_b e, var_b <- (1 - K_b) var_b';
      R <- R R_v^T
    not tracked: R <- R R_rel^T, v <- v', var_v <- var_v', var_b <- var_b', var_g <- var_g';
    w_prev <- w;
* a batch of frames gets its priors from the state at the batch start propagated by IMU-only
  steps (the device solves a batch's frames in parallel); after the batch the filter runs
  predict + update frame by frame on the results, each prior-weighted solution first taken back
  to its vision-only motion and covariance (``vision_only``; sigma^2 from the pose stats);
* the device: W_r adds W_r I to the rotation block of A7's Gauss-Newton and W_r delta to its
  gradient, W_t adds W_t I to the translation block and W_t (t_rel - t) to its gradient
  (``numpy_slam.refine``); an untracked frame with W_t > 0 is chained with the predicted
  [R_rel | t_rel] (``OracleTracker._advance``);
* a rig of several pairs (E_p = base_T_rect-left of pair p): pair p's prior is pair 0's moved into
  its camera, inv(E_p) E_0 T inv(E_0) E_p; the rig chains an untracked body frame with the
  prediction of the first pair with W_t > 0 moved to the body, (E_p T) inv(E_p) (``mul4``, as
  ``k_rig_prior``); the filter absorbs the rig's body motion moved into pair 0's camera,
  inv(E_0) M E_0, with the covariance Ad C Ad^T (Ad = the adjoint of inv(E_0)).
"""

from __future__ import annotations

import numpy as np
from scipy.spatial.transform import Rotation

GRAVITY = 9.81


class ImuFilter:
    def __init__(self, rect_R_imu: np.ndarray, acc_density: float = 2.553e-3, acc_random_walk: float = 1.0493e-4,
                 gyro_density: float = 8.27e-5, gyro_random_walk: float = 1e-8, rot_floor: float = 2e-4,
                 trans_floor: float = 1e-3, v0_sigma: float = 1.0, ba0_sigma: float = 0.05, bg0_sigma: float = 0.01,
                 lever: np.ndarray | None = None, accel: bool = True, vis_rot_floor: float = 1e-4):
        self.Ri = np.asarray(rect_R_imu, dtype=np.float64)
        self.na, self.rw = float(acc_density), float(acc_random_walk)
        self.ng, self.rwg = float(gyro_density), float(gyro_random_walk)
        self.rot_floor, self.floor, self.vis_floor = float(rot_floor), float(trans_floor), float(vis_rot_floor)
        self.v0_sigma, self.ba0_sigma, self.bg0_sigma = float(v0_sigma), float(ba0_sigma), float(bg0_sigma)
        self.r = np.zeros(3) if lever is None else np.asarray(lever, dtype=np.float64).reshape(3)
        self.accel = bool(accel)
        self.ready = False

    def start(self, accel: np.ndarray | None = None) -> None:
        self.R = np.eye(3)
        self.v = np.zeros(3)
        self.g = np.zeros(3)
        if self.accel:
            f = self.Ri @ np.asarray(accel, dtype=np.float64)
            self.g = -GRAVITY * f / np.linalg.norm(f)
        self.ba = np.zeros(3)
        self.bg = np.zeros(3)
        self.var_v = self.v0_sigma ** 2
        self.var_b = self.ba0_sigma ** 2
        self.var_g = self.bg0_sigma ** 2
        self.w_prev = None
        self.ready = True

    def state(self) -> tuple:
        return (self.R.copy(), self.v.copy(), self.ba.copy(), self.var_v, self.var_b, self.bg.copy(), self.var_g,
                None if self.w_prev is None else self.w_prev.copy())

    def set_state(self, st: tuple) -> None:
        self.R, self.v, self.ba, self.var_v, self.var_b = st[0].copy(), st[1].copy(), st[2].copy(), st[3], st[4]
        self.bg, self.var_g = st[5].copy(), st[6]
        self.w_prev = None if st[7] is None else st[7].copy()

    def predict(self, dt: float, gyro: np.ndarray, accel: np.ndarray | None) -> dict:
        gyro = np.asarray(gyro, dtype=np.float64)
        w = self.Ri @ (gyro - self.bg)
        r_rel = Rotation.from_rotvec(-w * dt).as_matrix()
        w_r = 1.0 / (self.ng ** 2 * dt + self.var_g * dt * dt + self.rot_floor ** 2)
        out = {"dt": dt, "gyro": gyro, "w": w, "R_rel": r_rel, "W_r": w_r, "t_rel": np.zeros(3), "W_t": 0.0}
        if not self.accel:
            return out
        alpha = np.zeros(3) if self.w_prev is None else (w - self.w_prev) / dt
        w_w, al_w, r_w = self.R @ w, self.R @ alpha, self.R @ self.r
        a_w = (self.R @ (self.Ri @ (np.asarray(accel, dtype=np.float64) - self.ba)) + self.g
               - np.cross(w_w, np.cross(w_w, r_w)) - np.cross(al_w, r_w))
        dp = self.v * dt + 0.5 * a_w * dt * dt
        c = self.R.T @ dp
        var_t = self.var_v * dt ** 2 + self.na ** 2 * dt ** 3 / 3.0 + self.var_b * dt ** 4 / 4.0 + self.floor ** 2
        out.update({"t_rel": -(r_rel @ c), "W_t": 1.0 / var_t, "v1": self.v + a_w * dt,
                    "var_v1": self.var_v + self.na ** 2 * dt + self.var_b * dt * dt})
        return out

    def update(self, pred: dict, status: int, t_rel: np.ndarray | None = None, cov: np.ndarray | None = None) -> None:
        dt = pred["dt"]
        var_g1 = self.var_g + self.rwg ** 2 * dt
        var_b1 = self.var_b + self.rw ** 2 * dt
        if status == 0:
            rv, tv = t_rel[:3, :3], t_rel[:3, 3]
            w_v = -Rotation.from_matrix(rv).as_rotvec() / dt
            z = pred["gyro"] - self.Ri.T @ w_v
            var_z = np.trace(cov[3:, 3:]) / 3.0 / dt ** 2 + self.ng ** 2 / dt + (self.vis_floor / dt) ** 2
            kg = var_g1 / (var_g1 + var_z)
            self.bg = self.bg + kg * (z - self.bg)
            self.var_g = (1.0 - kg) * var_g1
            if self.accel:
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
            if self.accel:
                self.v = pred["v1"]
                self.var_v = pred["var_v1"]
                self.var_b = var_b1
            self.var_g = var_g1
        self.w_prev = pred["w"]


def vision_only(T: np.ndarray, cov: np.ndarray, sigma2: float, prior: tuple) -> tuple:
    """The vision-only motion behind a prior-weighted A7 solution, for the gyroscope-bias update
    (a bias learnt from a rotation the gyro prior already pulled would never move): with
    H = sigma^2 C^-1 the solution's normal matrix in (rho, omega) and H_v = H - diag(W_t I, W_r I)
    the vision's part, one Gauss-Newton step from the solution on the vision alone,
    d = H_v^-1 [W_t (t - t_p); -W_r delta], delta = vee((R_p R^T - R R_p^T) / 2), applied as A7's
    left Cayley update (R_v = cay(d_omega) R, t_v = cay(d_omega) t + d_rho); its covariance
    sigma^2 H_v^-1.  Returns (T, C) unchanged when no prior acted or H_v is not positive definite."""
    from .numpy_slam import cayley

    r_p, w_r, t_p, w_t = prior
    if not sigma2 > 0.0 or not (w_r > 0.0 or w_t > 0.0):
        return T, cov
    h = sigma2 * np.linalg.inv(cov)
    hv = h.copy()
    hv[:3, :3] -= w_t * np.eye(3)
    hv[3:, 3:] -= w_r * np.eye(3)
    hv = 0.5 * (hv + hv.T)
    try:
        np.linalg.cholesky(hv)
    except np.linalg.LinAlgError:
        return T, cov
    R, t = T[:3, :3], T[:3, 3]
    a = r_p @ R.T
    delta = 0.5 * np.array([a[2, 1] - a[1, 2], a[0, 2] - a[2, 0], a[1, 0] - a[0, 1]])
    d = np.linalg.solve(hv, np.concatenate([w_t * (t - t_p), -w_r * delta]))
    ru = cayley(d[3:])
    out = np.eye(4)
    out[:3, :3] = ru @ R
    out[:3, 3] = ru @ t + d[:3]
    return out, sigma2 * np.linalg.inv(hv)


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


def _absorb(filt: ImuFilter, items: list, samples: list) -> None:
    """The filter absorbs a tracked batch: per frame (index, tracker result, prior)."""
    for i, r, pr in items:
        dt, gy, ac = samples[i]
        if dt is None:
            continue
        T, C = r["T"], r["cov"]
        if int(r["status"]) == 0 and pr is not None:
            T, C = vision_only(T, C, r["sigma2"], pr)
        filt.update(filt.predict(dt, gy, ac), int(r["status"]), T, C)


def lagged_priors(filt: ImuFilter, pending: list, batch_samples: list) -> list:
    """A batch's priors when the vision of the ``pending`` batches (tracked, not yet absorbed:
    lists of (index, ...) items, their samples first) is not in the filter yet: the state is
    coasted over their samples, then the batch's frames are predicted (HipSlamEngine with
    ``imu_prior_lag`` > 0: the prior of batch s uses the vision of batches <= s - 1 - lag)."""
    coast = [c for _, items, smp in pending for c in smp]
    return batch_priors(filt, coast + list(batch_samples))[len(coast):]


def run_sequence(tracker, frames: np.ndarray, samples: list, batch: int, filt: ImuFilter | None, lag: int = 0) -> list:
    """The engine's batch flow on the oracle tracker: ``samples[i]`` = (dt, gyro, accel) of frame
    i (dt None for the first).  With ``lag`` (``HipSlamConfig.imu_prior_lag``) the prior of batch
    s is computed before the vision of batches s - lag .. s - 1 is absorbed (they are coasted
    over), so that many batches may be in flight.  Returns the tracker's per-frame results."""
    results = []
    pending = []   # (batch number, [(i, result, prior)], [samples]) tracked, not yet absorbed
    for bi, b0 in enumerate(range(0, len(frames), batch)):
        idx = range(b0, min(b0 + batch, len(frames)))
        while filt is not None and pending and pending[0][0] <= bi - 1 - lag:
            _absorb(filt, pending.pop(0)[1], samples)
        if filt is not None and not filt.ready:
            filt.start(samples[b0][2])
        smp = [samples[i] for i in idx]
        priors = lagged_priors(filt, pending, smp) if filt is not None else [None] * len(idx)
        res = [tracker.step(frames[i, 0], frames[i, 1], prior=pr) for i, pr in zip(idx, priors)]
        pending.append((bi, list(zip(idx, res, priors)), smp))
        results += res
    return results


def _inv(t: np.ndarray) -> np.ndarray:
    out = np.eye(4)
    out[:3, :3] = t[:3, :3].T
    out[:3, 3] = -t[:3, :3].T @ t[:3, 3]
    return out


def _adjoint(t: np.ndarray) -> np.ndarray:
    r, tv = t[:3, :3], t[:3, 3]
    tx = np.array([[0.0, -tv[2], tv[1]], [tv[2], 0.0, -tv[0]], [-tv[1], tv[0], 0.0]])
    ad = np.zeros((6, 6))
    ad[:3, :3] = ad[3:, 3:] = r
    ad[:3, 3:] = tx @ r
    return ad


def pair_prior(prior: tuple, E: list, p: int) -> tuple:
    """Pair 0's prior moved into pair p's rectified-left camera: inv(E_p) E_0 T inv(E_0) E_p."""
    r0, w_r, t0, w_t = prior
    T = np.eye(4)
    T[:3, :3], T[:3, 3] = r0, t0
    if p:
        T = _inv(E[p]) @ E[0] @ T @ _inv(E[0]) @ E[p]
    return T[:3, :3], w_r, T[:3, 3], w_t


def run_rig_sequence(trackers: list, frames: np.ndarray, samples: list, batch: int, filt: ImuFilter, E: list,
                     cfg, lag: int = 0) -> list:
    """A multi-pair rig in the engine's batch flow: per batch the filter's pair-0 priors for every
    pair, each pair tracked, the rig pose over all pairs (``numpy_rig.rig_pose``), the rig chained
    (an untracked body frame with the first pair's W_t > 0 follows its prediction), and the filter
    absorbing the rig's motion in pair 0's camera.  Returns per frame {"status", "T_abs"} of the rig."""
    from .numpy_rig import inv_rigid, mul4, rig_pose

    Einv = [inv_rigid(e) for e in E]
    T_abs = np.eye(4)
    out = []
    pending = []   # (batch number, [(i, rig result)], [samples]) tracked, not yet absorbed

    def absorb(items):
        for i, res in items:
            dt, gy, ac = samples[i]
            if dt is None:
                continue
            st = int(res["status"])
            t0 = c0 = None
            if st == 0:
                t0 = _inv(E[0]) @ res["T"] @ E[0]
                ad = _adjoint(_inv(E[0]))
                c0 = ad @ res["cov"] @ ad.T
            filt.update(filt.predict(dt, gy, ac), st, t0, c0)

    for bi, b0 in enumerate(range(0, len(frames), batch)):
        idx = range(b0, min(b0 + batch, len(frames)))
        while pending and pending[0][0] <= bi - 1 - lag:
            absorb(pending.pop(0)[1])
        if not filt.ready:
            filt.start(samples[b0][2])
        smp = [samples[i] for i in idx]
        priors = lagged_priors(filt, pending, smp)
        results = []
        for i, pr in zip(idx, priors):
            outs = [trk.step(frames[i, 2 * q], frames[i, 2 * q + 1], prior=None if pr is None else pair_prior(pr, E, q))
                    for q, trk in enumerate(trackers)]
            if i == 0:
                res = {"status": 2, "T": np.eye(4), "cov": np.zeros((6, 6))}
            else:
                items = [{"status": o["status"], "T": o["T"], "corr": o.get("corr"),
                          "intr": (t.rect["fx"], t.rect["fy"], t.rect["cx"], t.rect["cy"])}
                         for o, t in zip(outs, trackers)]
                res = rig_pose(items, E, cfg)
            if res["status"] == 0:
                T_abs = T_abs @ inv_rigid(res["T"])
            elif pr is not None and pr[3] > 0.0:
                T = np.eye(4)
                T[:3, :3], T[:3, 3] = pr[0], pr[2]
                T_abs = T_abs @ inv_rigid(mul4(mul4(E[0], T), Einv[0]))
            results.append(res)
            out.append({"status": int(res["status"]), "T_abs": T_abs.copy()})
        pending.append((bi, list(zip(idx, results)), smp))
    return out
