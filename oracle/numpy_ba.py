"""Row A8 of SURVEY.md §8a — sliding-window local bundle adjustment, CPU restatement.

TEST INFRASTRUCTURE (see ``oracle/__init__.py``): the checker for the HIP back end's A8 kernels,
never imported by the product.  cuVSLAM's BA is closed, so this file *is* the
spec the kernels follow; parity against the reference is unpinned, like rows A2-A7.

Spec (shared with ``thor-slam_amd/csrc/k_ba.hip``):

* Keyframes: global frame g is a keyframe iff ``g % kf_interval == 0``; the window keeps the
  newest ``window`` keyframes in ``window`` slots (slot = keyframe number mod window).
* Observations of keyframe g: every valid keypoint k at its level-0 position
  ``u = (x + 0.5) * 2^l - 0.5`` (same for v); its stereo disparity (refined, NaN when unmatched)
  initialises new landmarks: ``Z = fx*B/d, X = (u-cx)Z/fx, Y = (v-cy)Z/fy`` in the camera,
  mapped to the world with the keyframe's pose.
* Association: ``link[k]`` = the keypoint of the previous keyframe reached by chaining the
  per-frame temporal matches back over the frames in between (-1 when the chain breaks).  A
  keypoint inherits its link's landmark; otherwise, with a finite disparity, it creates landmark
  ``slot * K + k``; else it has none.
* Eviction (a new keyframe reuses the oldest slot): every landmark homed in that slot moves to its
  observation in the oldest remaining keyframe that sees it (new id ``slot' * K + k'``, position
  copied, ids remapped in every keyframe); landmarks nobody else sees are dropped.
* Solve (``iters`` Gauss-Newton steps with Levenberg damping ``lam``), camera 0 = oldest keyframe
  held fixed (gauge):
    - cameras are ``cam_T_world`` (R, t); residual ``r = pi(R X + t) - z`` with the stereo row
      ``(fx (Xc - B) / Zc + cx) - (u - d)`` when the observation has a disparity (it fixes the scale
      a monocular window would leave free), zero otherwise;
    - ``J_c = dpi [I | -[Xc]x]`` (left update, translation first), ``J_p = dpi R``;
    - observations with an initial reprojection error > ``outlier_px`` or a non-positive depth are
      dropped; landmarks need >= 2 remaining observations;
    - ``S = blockdiag(U_c + lam I) - sum_i sum_{o,o' in i} W_o V_i^-1 W_o'^T``,
      ``b = -g_c + sum_i sum_{o in i} W_o V_i^-1 g_p,i`` with ``V_i = sum J_p^T J_p + lam I``;
    - ``S' dc = b'`` without camera 0 (Cholesky), ``dp_i = V_i^-1 (-g_p,i - sum_o W_o^T dc_o)``;
    - cameras ``R <- cayley(w) R, t <- cayley(w) t + rho``; points ``X += dp``.
* IMU rotation factors (optional): keyframe g may carry the gyro-integrated rotation ``M`` from the
  previous keyframe's camera to its own (frame g - kf_interval points to frame g) with a weight
  ``w`` (1 / rad^2, 0 = none).  Between window-consecutive keyframes (c - 1, c) whose later one
  carries a factor, with ``Q = R_c R_{c-1}^T`` and ``e = vee((A - A^T) / 2)``, ``A = M^T Q``: the
  residual e has Jacobians ``Q^T`` on camera c's rotation and ``-I`` on camera c - 1's (left
  updates), so ``S_cc += w I``, ``S_{c-1,c-1} += w I``, ``S_{c,c-1} += -w Q`` (rotation blocks),
  ``b_c -= w Q e``, ``b_{c-1} += w e``; camera 0's rows drop with the gauge.
* Inertial factors (tightly coupled, optional; SURVEY.md §8f item 2 with the biases and random
  walks of ``launch/thor_visual_slam.launch.py:50-53,88-93``): keyframe g may carry the IMU
  preintegration from the previous keyframe (``preintegrate``, record layout at ``INE_N``) and an
  initial world velocity of its camera.  Every window keyframe c carries the states y_c = (v_c,
  ba_c, bg_c): its camera's world velocity and the accelerometer / gyroscope biases (IMU axes)
  over the interval that starts at it.  ``set_inertial``: world gravity gw and priors (ba0, wb),
  (bg0, wg) on the oldest keyframe's biases.  Between window-consecutive keyframes (i, j) =
  (c - 1, c) whose later one carries a factor, with R_i the cam_T_world rotation, p the camera
  centres, dba = ba_i - ba_lin, dbg = bg_i - bg_lin, Q = R_j R_i^T and A = M^T Q:
      r_v  = R_i (v_j - v_i - gw dt) - (dv + Jv dba + Jvg dbg)            weight wv
      r_p  = R_i (p_j - p_i - v_i dt - gw dt^2 / 2) - (dp + Jp dba + Jpg dbg)   wp
      r_R  = vee((A - A^T) / 2) + JRe dbg                                 wR (0: no rotation rows)
      r_ba = ba_j - ba_i,   r_bg = bg_j - bg_i                            w_ra, w_rg (random walks)
  with the Jacobians of ``inertial_jacobian`` (left camera updates (rho, omega): d(R_i u)/d omega_i
  = -[R_i u]x, dp/d rho = -R_wc; the rotation rows take the IMU rotation factor's Q^T / -I).  With
  y = (y_0 .. y_{n-1}) (9 per keyframe) the normal equations [[S + lam I, Hxy], [Hyx, Hyy]] (Hyy
  with lam I and the priors on y_0's biases) are reduced to the cameras, S' = S - Hxy Hyy^-1 Hyx,
  b' = b - Hxy Hyy^-1 b_y (camera 0's rows dropped first); after the camera solve
  dy = Hyy^-1 (b_y - Hyx dc) updates every keyframe's velocity and biases.  A new keyframe's biases
  start at its record's (ba_lin, bg_lin), or the previous keyframe's without a record.  A window
  with no inertial factor skips all of it (the solve is the visual one, bit for bit).
"""

from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from .numpy_slam import cayley, level0_coords

# inertial factor record per slot (k_ba.hip TS_BA_INE): dv 0-2, dp 3-5, Jv 6-14 and Jp 15-23
# (d/d ba, row-major 3x3), ba_lin 24-26, dt 27, wv 28 (0 = no factor), wp 29, wR 30 (rotation
# rows), w_ra 31 (accelerometer-bias random walk), M 32-40 (the gyro rotation, camera i points ->
# camera j), JRe 41-49 (d r_R / d bg), Jvg 50-58 and Jpg 59-67 (d/d bg), bg_lin 68-70, w_rg 71
# (gyroscope-bias random walk), 72-79 unused
INE_N = 80
INE_Y = 9   # states per keyframe: v, ba, bg


def _exp_so3(w: np.ndarray) -> np.ndarray:
    th = float(np.linalg.norm(w))
    K = np.array([[0.0, -w[2], w[1]], [w[2], 0.0, -w[0]], [-w[1], w[0], 0.0]])
    if th < 1e-12:
        return np.eye(3) + K
    return np.eye(3) + np.sin(th) / th * K + (1.0 - np.cos(th)) / (th * th) * (K @ K)


def _jr_so3(w: np.ndarray) -> np.ndarray:
    """Right Jacobian of SO(3): I - (1 - cos t) / t^2 [w]x + (t - sin t) / t^3 [w]x^2 (series
    below t = 1e-4)."""
    th = float(np.linalg.norm(w))
    K = np.array([[0.0, -w[2], w[1]], [w[2], 0.0, -w[0]], [-w[1], w[0], 0.0]])
    if th < 1e-4:
        return np.eye(3) - 0.5 * K + (K @ K) / 6.0
    return np.eye(3) - (1.0 - np.cos(th)) / (th * th) * K + (th - np.sin(th)) / (th * th * th) * (K @ K)


def preintegrate(samples: list, rect_R_imu: np.ndarray, bg: np.ndarray, ba: np.ndarray,
                 lever: np.ndarray | None = None, w_prev: np.ndarray | None = None,
                 acc_density: float = 2.553e-3, v_floor: float = 1e-2, p_floor: float = 1e-3,
                 gyro_density: float = 0.0, r_floor: float = 0.0, acc_rw: float = 0.0, gyro_rw: float = 0.0,
                 ba_floor: float = 1e-3, bg_floor: float = 1e-3) -> np.ndarray:
    """The inertial factor record (INE_N doubles) of the frame intervals ``samples`` = [(dt, gyro,
    accel)] (IMU axes) from one keyframe to the next, in the first keyframe's camera axes: per
    interval w = Ri (gyro - bg) (camera axes), alpha = (w - w_prev) / dt (0 for the first interval
    without ``w_prev``), the camera's specific force a = Ri (accel - ba) - w x (w x r) - alpha x r
    (r = the IMU's position in the camera, as ``numpy_imu.ImuFilter``), then
        dp += dv dt + dR a dt^2 / 2,   Jp += Jv dt - dR Ri dt^2 / 2,
        dv += dR a dt,                 Jv += -dR Ri dt,
        Jpg += Jvg dt - dR [a]x JR dt^2 / 2,   Jvg += -dR [a]x JR dt,
        JR <- exp(w dt)^T JR - Jr(w dt) Ri dt,   dR <- dR exp([w dt]x)
    (the gyroscope bias enters through the rotation; the lever-arm terms' own dependence on it is
    left out), M = dR^T, JRe = dR JR; weights over the total T: wv = 1 / (n_a^2 T + v_floor^2),
    wp = 1 / (n_a^2 T^3 / 3 + p_floor^2), wR = 1 / (n_g^2 T + r_floor^2) (0 when n_g = 0), the
    bias random walks w_ra = 1 / (s_a^2 T + ba_floor^2), w_rg = 1 / (s_g^2 T + bg_floor^2) (0 when
    s = 0)."""
    Ri = np.asarray(rect_R_imu, dtype=np.float64)
    r = np.zeros(3) if lever is None else np.asarray(lever, dtype=np.float64)
    bg = np.asarray(bg, dtype=np.float64)
    ba = np.asarray(ba, dtype=np.float64)
    dR, dv, dp = np.eye(3), np.zeros(3), np.zeros(3)
    Jv, Jp, Jvg, Jpg, JR = (np.zeros((3, 3)) for _ in range(5))
    T = 0.0
    wp = None if w_prev is None else np.asarray(w_prev, dtype=np.float64)
    for dt, gyro, accel in samples:
        w = Ri @ (np.asarray(gyro, dtype=np.float64) - bg)
        al = np.zeros(3) if wp is None else (w - wp) / dt
        a = Ri @ (np.asarray(accel, dtype=np.float64) - ba) - np.cross(w, np.cross(w, r)) - np.cross(al, r)
        Ra = dR @ _skew(a) @ JR
        dp = dp + dv * dt + 0.5 * (dR @ a) * dt * dt
        Jp = Jp + Jv * dt - 0.5 * (dR @ Ri) * dt * dt
        Jpg = Jpg + Jvg * dt - 0.5 * Ra * dt * dt
        dv = dv + (dR @ a) * dt
        Jv = Jv - (dR @ Ri) * dt
        Jvg = Jvg - Ra * dt
        E = _exp_so3(w * dt)
        JR = E.T @ JR - _jr_so3(w * dt) @ Ri * dt
        dR = dR @ E
        T += dt
        wp = w
    out = np.zeros(INE_N)
    out[0:3], out[3:6], out[6:15], out[15:24], out[24:27] = dv, dp, Jv.reshape(9), Jp.reshape(9), ba
    out[27] = T
    out[28] = 1.0 / (acc_density ** 2 * T + v_floor ** 2)
    out[29] = 1.0 / (acc_density ** 2 * T ** 3 / 3.0 + p_floor ** 2)
    out[30] = 1.0 / (gyro_density ** 2 * T + r_floor ** 2) if gyro_density > 0.0 else 0.0
    out[31] = 1.0 / (acc_rw ** 2 * T + ba_floor ** 2) if acc_rw > 0.0 else 0.0
    out[32:41] = dR.T.reshape(9)
    out[41:50] = (dR @ JR).reshape(9)
    out[50:59], out[59:68], out[68:71] = Jvg.reshape(9), Jpg.reshape(9), bg
    out[71] = 1.0 / (gyro_rw ** 2 * T + bg_floor ** 2) if gyro_rw > 0.0 else 0.0
    return out


def inertial_residual(f: np.ndarray, Rcw_i: np.ndarray, tcw_i: np.ndarray, Rcw_j: np.ndarray, tcw_j: np.ndarray,
                      v_i: np.ndarray, v_j: np.ndarray, bias_i: np.ndarray, bias_j: np.ndarray,
                      gw: np.ndarray) -> np.ndarray:
    """(r_v, r_p, r_R, r_ba, r_bg) (15) of one inertial factor record at the cameras cam_T_world
    i, j, velocities and biases (ba, bg) = bias[0:3], bias[3:6]."""
    dt = f[27]
    dba = bias_i[0:3] - f[24:27]
    dbg = bias_i[3:6] - f[68:71]
    p_i, p_j = -Rcw_i.T @ tcw_i, -Rcw_j.T @ tcw_j
    uv = v_j - v_i - gw * dt
    up = p_j - p_i - v_i * dt - 0.5 * gw * dt * dt
    rv = Rcw_i @ uv - (f[0:3] + f[6:15].reshape(3, 3) @ dba + f[50:59].reshape(3, 3) @ dbg)
    rp = Rcw_i @ up - (f[3:6] + f[15:24].reshape(3, 3) @ dba + f[59:68].reshape(3, 3) @ dbg)
    A = f[32:41].reshape(3, 3).T @ (Rcw_j @ Rcw_i.T)
    rR = 0.5 * np.array([A[2, 1] - A[1, 2], A[0, 2] - A[2, 0], A[1, 0] - A[0, 1]]) + f[41:50].reshape(3, 3) @ dbg
    return np.concatenate([rv, rp, rR, bias_j[0:3] - bias_i[0:3], bias_j[3:6] - bias_i[3:6]])


def inertial_weights(f: np.ndarray) -> np.ndarray:
    return np.array([f[28]] * 3 + [f[29]] * 3 + [f[30]] * 3 + [f[31]] * 3 + [f[71]] * 3)


def inertial_system(st, slots: list[int], Rs: np.ndarray, ts: np.ndarray, S: np.ndarray, b: np.ndarray) -> tuple | None:
    """``KeyframeWindow.inertial_terms`` for any window state ``st`` carrying ``ine``, ``vel``,
    ``bias``, ``ine_cfg`` and ``p.lam`` (a pair window, or a rig's body window with the body poses
    as the cameras)."""
    n = len(slots)
    fs = [c for c in range(1, n) if st.ine[slots[c]][28] > 0.0]
    if not fs:
        return None
    gw, ba0, wb, bg0, wg = st.ine_cfg
    my = INE_Y * n
    Hxy = np.zeros((6 * n, my))
    Hyy = np.zeros((my, my))
    by = np.zeros(my)
    for c in fs:
        f = st.ine[slots[c]]
        i, j = c - 1, c
        vi, vj = st.vel[slots[i]], st.vel[slots[j]]
        bi, bj = st.bias[slots[i]], st.bias[slots[j]]
        r = inertial_residual(f, Rs[i], ts[i], Rs[j], ts[j], vi, vj, bi, bj, gw)
        J = inertial_jacobian(f, Rs[i], ts[i], Rs[j], ts[j], vi, vj, gw)
        Wd = inertial_weights(f)
        xc = list(range(6 * i, 6 * i + 6)) + list(range(6 * j, 6 * j + 6))
        yc = list(range(INE_Y * i, INE_Y * i + INE_Y)) + list(range(INE_Y * j, INE_Y * j + INE_Y))
        Jx, Jy = J[:, :12], J[:, 12:]
        WJx, WJy = Wd[:, None] * Jx, Wd[:, None] * Jy
        S[np.ix_(xc, xc)] += Jx.T @ WJx
        b[xc] -= Jx.T @ (Wd * r)
        Hxy[np.ix_(xc, yc)] += Jx.T @ WJy
        Hyy[np.ix_(yc, yc)] += Jy.T @ WJy
        by[yc] -= Jy.T @ (Wd * r)
    b0 = st.bias[slots[0]]   # the priors on the oldest keyframe's biases
    Hyy[3:6, 3:6] += wb * np.eye(3)
    by[3:6] -= wb * (b0[0:3] - ba0)
    Hyy[6:9, 6:9] += wg * np.eye(3)
    by[6:9] -= wg * (b0[3:6] - bg0)
    Hyy += st.p.lam * np.eye(my)
    return Hxy, Hyy, by


def inertial_step(st, slots: list[int], S: np.ndarray, b: np.ndarray, ine: tuple) -> np.ndarray:
    """Solve the damped camera system ``S`` (6n, lam included), ``b`` with the velocity / bias
    unknowns of ``ine`` = (Hxy, Hyy, b_y) eliminated (camera 0 = gauge); apply dy to ``st``'s
    velocities and biases; return the 6n camera step (zeros for camera 0)."""
    n = len(slots)
    Hxy, Hyy, by = ine
    Hx = Hxy[6:]
    Z = np.linalg.solve(Hyy, Hx.T)          # Hyy^-1 Hyx
    zb = np.linalg.solve(Hyy, by)
    dc = np.zeros(6 * n)
    dc[6:] = np.linalg.solve(S[6:, 6:] - Hx @ Z, b[6:] - Hx @ zb)
    dy = zb - Z @ dc[6:]
    for c in range(n):
        y = dy[INE_Y * c:INE_Y * c + INE_Y]
        st.vel[slots[c]] = st.vel[slots[c]] + y[0:3]
        st.bias[slots[c]] = st.bias[slots[c]] + y[3:9]
    return dc


def inertial_jacobian(f: np.ndarray, Rcw_i: np.ndarray, tcw_i: np.ndarray, Rcw_j: np.ndarray, tcw_j: np.ndarray,
                      v_i: np.ndarray, v_j: np.ndarray, gw: np.ndarray) -> np.ndarray:
    """15 x 30 Jacobian of ``inertial_residual``: columns rho_i, omega_i, rho_j, omega_j (left
    camera updates), then y_i = (v_i, ba_i, bg_i), y_j = (v_j, ba_j, bg_j)."""
    dt = f[27]
    p_i, p_j = -Rcw_i.T @ tcw_i, -Rcw_j.T @ tcw_j
    uv = v_j - v_i - gw * dt
    up = p_j - p_i - v_i * dt - 0.5 * gw * dt * dt
    J = np.zeros((15, 30))
    J[0:3, 3:6] = -_skew(Rcw_i @ uv)
    J[0:3, 12:15] = -Rcw_i
    J[0:3, 15:18] = -f[6:15].reshape(3, 3)
    J[0:3, 18:21] = -f[50:59].reshape(3, 3)
    J[0:3, 21:24] = Rcw_i
    J[3:6, 0:3] = np.eye(3)
    J[3:6, 3:6] = -_skew(Rcw_i @ up)
    J[3:6, 6:9] = -Rcw_i @ Rcw_j.T
    J[3:6, 12:15] = -Rcw_i * dt
    J[3:6, 15:18] = -f[15:24].reshape(3, 3)
    J[3:6, 18:21] = -f[59:68].reshape(3, 3)
    J[6:9, 3:6] = -np.eye(3)
    J[6:9, 9:12] = (Rcw_j @ Rcw_i.T).T
    J[6:9, 18:21] = f[41:50].reshape(3, 3)
    J[9:12, 15:18], J[9:12, 24:27] = -np.eye(3), np.eye(3)
    J[12:15, 18:21], J[12:15, 27:30] = -np.eye(3), np.eye(3)
    return J


@dataclass
class BAParams:
    window: int = 10
    kf_interval: int = 5
    iters: int = 5
    lam: float = 1.0
    outlier_px: float = 3.0


def chain_links(temporal_maps: list[np.ndarray]) -> np.ndarray:
    """Compose per-frame temporal maps (newest first: frame g, g-1, ...) into keypoint -> keypoint
    of the frame before the last map (-1 where any step is unmatched)."""
    idx = np.arange(temporal_maps[0].size)
    out = idx.copy()
    for tm in temporal_maps:
        ok = out >= 0
        out = np.where(ok, tm[np.where(ok, out, 0)], -1)
    return out


class KeyframeWindow:
    """The keyframe slots, landmark table and solver of one stereo pair (restated spec)."""

    def __init__(self, K: int, intr, params: BAParams):
        self.K = K
        self.fx, self.fy, self.cx, self.cy, self.fxb = intr
        self.p = params
        W = params.window
        self.frame = np.full(W, -1, dtype=np.int64)       # global frame of each slot (-1 = empty)
        self.T_cw = np.tile(np.eye(4), (W, 1, 1))
        self.u = np.full((W, K), np.nan)
        self.v = np.full((W, K), np.nan)
        self.d = np.full((W, K), np.nan)
        self.lm = np.full((W, K), -1, dtype=np.int64)
        self.X = np.zeros((W * K, 3))
        self.imu_M = np.tile(np.eye(3), (W, 1, 1))   # IMU rotation from the previous keyframe
        self.imu_w = np.zeros(W)                     # its weight (0 = no factor)
        self.ine = np.zeros((W, INE_N))              # inertial factor from the previous keyframe
        self.vel = np.zeros((W, 3))                  # world velocity of the keyframe's camera
        self.bias = np.zeros((W, 6))                 # its accelerometer and gyroscope biases (IMU axes)
        # gravity (world), accelerometer-bias prior and weight, gyroscope-bias prior and weight
        self.ine_cfg = (np.zeros(3), np.zeros(3), 0.0, np.zeros(3), 0.0)
        self.n_kf = 0

    # -- window bookkeeping --------------------------------------------------------------------
    def order(self) -> list[int]:
        """Occupied slots, oldest keyframe first."""
        occ = [s for s in range(self.p.window) if self.frame[s] >= 0]
        return sorted(occ, key=lambda s: self.frame[s])

    def _evict(self, slot: int) -> None:
        K = self.K
        lo, hi = slot * K, slot * K + K
        rest = [s for s in self.order() if s != slot]
        remap = np.full(K, -1, dtype=np.int64)
        for s in rest:                       # oldest remaining keyframe first
            lm = self.lm[s]
            hit = (lm >= lo) & (lm < hi)
            for k in np.nonzero(hit)[0]:
                old = lm[k] - lo
                if remap[old] < 0:
                    remap[old] = s * K + k
                    self.X[s * K + k] = self.X[lm[k]]
        for s in rest:
            lm = self.lm[s]
            hit = (lm >= lo) & (lm < hi)
            lm[hit] = remap[lm[hit] - lo]
        self.lm[slot] = -1
        self.frame[slot] = -1

    def add_keyframe(self, g: int, T_cw: np.ndarray, u: np.ndarray, v: np.ndarray, disp: np.ndarray,
                     link: np.ndarray | None, imu: tuple | None = None, ine: tuple | None = None) -> int:
        """Insert keyframe g (u, v level-0 observations, NaN = invalid; disp refined, NaN = none;
        link into the previous keyframe or None for the first; imu = (M, w) the IMU rotation
        factor from the previous keyframe, or None; ine = (record, v0) the inertial factor from
        the previous keyframe (``preintegrate``) and the camera's initial world velocity, or
        None: no factor, velocity 0)."""
        K = self.K
        slot = self.n_kf % self.p.window
        prev = self.order()[-1] if self.n_kf else -1
        if self.frame[slot] >= 0:
            self._evict(slot)
        self.frame[slot] = g
        self.T_cw[slot] = T_cw
        self.imu_M[slot], self.imu_w[slot] = (np.eye(3), 0.0) if imu is None else (np.asarray(imu[0], float), float(imu[1]))
        self.ine[slot] = 0.0 if ine is None else np.asarray(ine[0], dtype=np.float64)
        self.vel[slot] = 0.0 if ine is None else np.asarray(ine[1], dtype=np.float64)
        self.bias[slot] = new_keyframe_bias(self.ine[slot], self.bias, prev)
        self.u[slot], self.v[slot] = u, v
        self.d[slot] = np.where(np.isfinite(disp) & (disp > 0), disp, np.nan)
        valid = np.isfinite(u)
        lm = np.full(K, -1, dtype=np.int64)
        if link is not None and prev >= 0:
            has = valid & (link >= 0)
            inh = np.where(has, self.lm[prev][np.where(has, link, 0)], -1)
            lm = np.where(has, inh, -1)
        new = valid & (lm < 0) & np.isfinite(disp) & (disp > 0)
        ks = np.nonzero(new)[0]
        lm[ks] = slot * K + ks
        if ks.size:
            z = self.fxb / disp[ks]
            xc = np.stack([(u[ks] - self.cx) * z / self.fx, (v[ks] - self.cy) * z / self.fy, z], axis=1)
            R, t = T_cw[:3, :3], T_cw[:3, 3]
            self.X[slot * K + ks] = (xc - t) @ R       # R^T (xc - t)
        self.lm[slot] = lm
        self.n_kf += 1
        return slot

    # -- solve -----------------------------------------------------------------------------------
    def observations(self):
        """(camera index, landmark id, u, v, d) of every observation, cameras oldest first."""
        cams, lms, us, vs, ds = [], [], [], [], []
        for ci, s in enumerate(self.order()):
            k = np.nonzero(self.lm[s] >= 0)[0]
            cams.append(np.full(k.size, ci))
            lms.append(self.lm[s][k])
            us.append(self.u[s][k])
            vs.append(self.v[s][k])
            ds.append(self.d[s][k])
        return (np.concatenate(cams), np.concatenate(lms), np.concatenate(us), np.concatenate(vs),
                np.concatenate(ds))

    def _project(self, R, t, X):
        xc = np.einsum("nij,nj->ni", R, X) + t
        return xc, self.fx * xc[:, 0] / xc[:, 2] + self.cx, self.fy * xc[:, 1] / xc[:, 2] + self.cy

    def prepare(self, T: np.ndarray) -> dict | None:
        """Observation set of a solve at cameras ``T`` (cam_T_world per occupied slot, oldest
        first): the outlier / depth gate at the current estimate, then >= 2 observations per
        landmark.  None when fewer than two keyframes are occupied."""
        p = self.p
        if T.shape[0] < 2:
            return None
        cam, lm, uo, vo, do = self.observations()
        xc, pu, pv = self._project(T[cam, :3, :3], T[cam, :3, 3], self.X[lm])
        keep = (xc[:, 2] > 0) & ((pu - uo) ** 2 + (pv - vo) ** 2 <= p.outlier_px * p.outlier_px)
        cnt = np.bincount(lm[keep], minlength=self.X.shape[0])
        keep &= cnt[lm] >= 2
        cam, lm, uo, vo, do = cam[keep], lm[keep], uo[keep], vo[keep], do[keep]
        st = np.isfinite(do)                           # observations with a stereo row
        ur = np.where(st, uo - np.where(st, do, 0.0), 0.0)
        ids, li = np.unique(lm, return_inverse=True)   # compact landmark index per observation
        return {"n": T.shape[0], "cam": cam, "lm": lm, "uo": uo, "vo": vo, "st": st, "ur": ur, "ids": ids, "li": li,
                "X": self.X[ids].copy()}

    def linearize(self, ob: dict, Rs: np.ndarray, ts: np.ndarray) -> dict:
        """One Gauss-Newton linearisation at cameras (Rs, ts) and landmarks ob["X"]: the reduced
        camera system WITHOUT the camera damping, S = blockdiag(U_c) - sum W_o V_i^-1 W_o'^T and
        b = -g_c + sum W_o V_i^-1 g_p,i (6n x 6n, 6n), and what the back substitution needs."""
        p = self.p
        n, cam, li, uo, vo, st, ur, X = ob["n"], ob["cam"], ob["li"], ob["uo"], ob["vo"], ob["st"], ob["ur"], ob["X"]
        L = ob["ids"].size
        fx, fy = self.fx, self.fy
        base = self.fxb / self.fx
        R = Rs[cam]
        xc = np.einsum("nij,nj->ni", R, X[li]) + ts[cam]
        iz = 1.0 / xc[:, 2]
        r3 = np.where(st, fx * (xc[:, 0] - base) * iz + self.cx - ur, 0.0)
        r = np.stack([fx * xc[:, 0] * iz + self.cx - uo, fy * xc[:, 1] * iz + self.cy - vo, r3], axis=1)
        dpi = np.zeros((cam.size, 3, 3))
        dpi[:, 0, 0] = fx * iz
        dpi[:, 0, 2] = -fx * xc[:, 0] * iz * iz
        dpi[:, 1, 1] = fy * iz
        dpi[:, 1, 2] = -fy * xc[:, 1] * iz * iz
        dpi[:, 2, 0] = np.where(st, fx * iz, 0.0)
        dpi[:, 2, 2] = np.where(st, -fx * (xc[:, 0] - base) * iz * iz, 0.0)
        skew = np.zeros((cam.size, 3, 3))
        skew[:, 0, 1], skew[:, 0, 2] = -xc[:, 2], xc[:, 1]
        skew[:, 1, 0], skew[:, 1, 2] = xc[:, 2], -xc[:, 0]
        skew[:, 2, 0], skew[:, 2, 1] = -xc[:, 1], xc[:, 0]
        Jc = np.concatenate([dpi, -np.einsum("nij,njk->nik", dpi, skew)], axis=2)   # n x 3 x 6
        Jp = np.einsum("nij,njk->nik", dpi, R)                                        # n x 3 x 3
        U = np.zeros((n, 6, 6))
        gc = np.zeros((n, 6))
        np.add.at(U, cam, np.einsum("nki,nkj->nij", Jc, Jc))
        np.add.at(gc, cam, np.einsum("nki,nk->ni", Jc, r))
        V = np.tile(np.eye(3) * p.lam, (L, 1, 1))
        gp = np.zeros((L, 3))
        np.add.at(V, li, np.einsum("nki,nkj->nij", Jp, Jp))
        np.add.at(gp, li, np.einsum("nki,nk->ni", Jp, r))
        Vinv = np.linalg.inv(V)
        Wo = np.einsum("nki,nkj->nij", Jc, Jp)                                        # n x 6 x 3
        S = np.zeros((6 * n, 6 * n))
        for c in range(n):
            S[6 * c:6 * c + 6, 6 * c:6 * c + 6] += U[c]
        b = -gc.reshape(-1).copy()
        WV = np.einsum("nij,njk->nik", Wo, Vinv[li])                                   # W_o V_i^-1
        np.add.at(b.reshape(n, 6), cam, np.einsum("nij,nj->ni", WV, gp[li]))
        order = np.argsort(li, kind="stable")
        starts = np.searchsorted(li[order], np.arange(L + 1))
        for i in range(L):
            obs = order[starts[i]:starts[i + 1]]
            for a in obs:
                for bb in obs:
                    ca, cb = cam[a], cam[bb]
                    S[6 * ca:6 * ca + 6, 6 * cb:6 * cb + 6] -= WV[a] @ Wo[bb].T
        return {"S": S, "b": b, "Wo": Wo, "gp": gp, "Vinv": Vinv}

    @staticmethod
    def landmark_update(ob: dict, lin: dict, dcc: np.ndarray) -> np.ndarray:
        """dp_i = V_i^-1 (-g_p,i - sum_o W_o^T dc_o) for camera updates dcc (n x 6)."""
        rhs = -lin["gp"].copy()
        np.add.at(rhs, ob["li"], -np.einsum("nji,nj->ni", lin["Wo"], dcc[ob["cam"]]))
        return np.einsum("lij,lj->li", lin["Vinv"], rhs)

    def imu_terms(self, slots: list[int], Rs: np.ndarray, S: np.ndarray, b: np.ndarray) -> None:
        """The IMU rotation factors between window-consecutive keyframes, into S and b in place."""
        for c in range(1, len(slots)):
            w = self.imu_w[slots[c]]
            if not w > 0.0:
                continue
            Q = Rs[c] @ Rs[c - 1].T
            A = self.imu_M[slots[c]].T @ Q
            e = 0.5 * np.array([A[2, 1] - A[1, 2], A[0, 2] - A[2, 0], A[1, 0] - A[0, 1]])
            rc, rp = 6 * c + 3, 6 * (c - 1) + 3
            S[rc:rc + 3, rc:rc + 3] += w * np.eye(3)
            S[rp:rp + 3, rp:rp + 3] += w * np.eye(3)
            S[rc:rc + 3, rp:rp + 3] -= w * Q
            S[rp:rp + 3, rc:rc + 3] -= w * Q.T
            b[rc:rc + 3] -= w * (Q @ e)
            b[rp:rp + 3] += w * e

    def set_inertial(self, gw: np.ndarray, ba0: np.ndarray, wb: float, bg0: np.ndarray | None = None,
                     wg: float = 0.0) -> None:
        """World gravity and the priors (value, weight) on the oldest keyframe's accelerometer and
        gyroscope biases for the next solves."""
        self.ine_cfg = _ine_cfg(gw, ba0, wb, bg0, wg)

    def inertial_terms(self, slots: list[int], Rs: np.ndarray, ts: np.ndarray, S: np.ndarray,
                       b: np.ndarray) -> tuple | None:
        """The inertial factors into S and b (camera-camera parts, in place) and the velocity /
        bias system (Hxy 6n x (3n+3), Hyy with lam I and the bias prior, b_y); None without
        factors."""
        return inertial_system(self, slots, Rs, ts, S, b)

    def inertial_solve(self, slots: list[int], S: np.ndarray, b: np.ndarray, ine: tuple) -> np.ndarray:
        """The camera step (gauge camera 0 dropped) with the velocity / bias unknowns eliminated,
        and their own step applied to the window's velocities and bias."""
        return inertial_step(self, slots, S, b, ine)

    def solve(self) -> dict:
        p = self.p
        slots = self.order()
        n = len(slots)
        T = self.T_cw[slots]
        ob = self.prepare(T)
        if ob is None:
            return {"n_obs": 0, "n_lm": 0}
        Rs, ts = T[:, :3, :3].copy(), T[:, :3, 3].copy()
        for _ in range(p.iters):
            lin = self.linearize(ob, Rs, ts)
            self.imu_terms(slots, Rs, lin["S"], lin["b"])
            ine = self.inertial_terms(slots, Rs, ts, lin["S"], lin["b"])
            S = lin["S"] + p.lam * np.eye(6 * n)
            dc = np.zeros(6 * n)
            if ine is None:
                dc[6:] = np.linalg.solve(S[6:, 6:], lin["b"][6:])
            else:
                dc = self.inertial_solve(slots, S, lin["b"], ine)
            dcc = dc.reshape(n, 6)
            dp = self.landmark_update(ob, lin, dcc)
            for c in range(1, n):
                ru = cayley(dcc[c, 3:])
                Rs[c] = ru @ Rs[c]
                ts[c] = ru @ ts[c] + dcc[c, :3]
            ob["X"] = ob["X"] + dp
        for c, s in enumerate(slots):
            self.T_cw[s, :3, :3], self.T_cw[s, :3, 3] = Rs[c], ts[c]
        return self._finish(ob, Rs, ts)

    def _finish(self, ob: dict, Rs: np.ndarray, ts: np.ndarray) -> dict:
        cam, li, uo, vo = ob["cam"], ob["li"], ob["uo"], ob["vo"]
        self.X[ob["ids"]] = ob["X"]
        xc, pu, pv = self._project(Rs[cam], ts[cam], ob["X"][li])
        rms = float(np.sqrt(np.mean((pu - uo) ** 2 + (pv - vo) ** 2))) if cam.size else 0.0
        return {"n_obs": int(cam.size), "n_lm": int(ob["ids"].size), "rms_px": rms}


def _ine_cfg(gw, ba0, wb, bg0, wg) -> tuple:
    return (np.asarray(gw, dtype=np.float64).copy(), np.asarray(ba0, dtype=np.float64).copy(), float(wb),
            np.zeros(3) if bg0 is None else np.asarray(bg0, dtype=np.float64).copy(), float(wg))


def new_keyframe_bias(record: np.ndarray, bias: np.ndarray, prev: int) -> np.ndarray:
    """A new keyframe's (ba, bg): its record's linearisation point, or the previous keyframe's
    biases without a record (zeros for the first keyframe)."""
    if record[28] > 0.0:
        return np.concatenate([record[24:27], record[68:71]])
    return bias[prev].copy() if prev >= 0 else np.zeros(6)


def _skew(t: np.ndarray) -> np.ndarray:
    return np.array([[0.0, -t[2], t[1]], [t[2], 0.0, -t[0]], [-t[1], t[0], 0.0]])


def adjoint_rl(T: np.ndarray) -> np.ndarray:
    """Adjoint of rigid T = [R | t] for left perturbations in (rho, omega) order:
    (I + (Ad d)^) T = T (I + d^), Ad = [[R, [t]x R], [0, R]]."""
    R, t = T[:3, :3], T[:3, 3]
    A = np.zeros((6, 6))
    A[:3, :3] = R
    A[:3, 3:] = _skew(t) @ R
    A[3:, 3:] = R
    return A


class RigKeyframeWindow:
    """The rig-level A8 window: ONE body pose per keyframe (body_T_world, slots shared by the
    pairs) and each pair's observations and landmarks in its own ``KeyframeWindow`` whose cameras
    are functions of the body poses, cam_T_world_p = E_p^-1 B (E_p = base_T_rect-left).

    Solve (rig extension of ``KeyframeWindow.solve``; spec shared with k_ba.hip's rig kernels):
    a left body update B <- (I + d^) B moves pair p's camera by Ad_p d, Ad_p = adjoint_rl(E_p^-1),
    so each pair's reduced system (S_p, b_p) at its cameras E_p^-1 B — undamped, landmark damping
    inside as in the one-pair solve — enters the body system as
        S = sum_p Ad_p^T S_p Ad_p (6x6 blocks, pairs in order) + lam I,   b = sum_p Ad_p^T b_p;
    body 0 (oldest keyframe) is the gauge; S' dB = b' by Cholesky; each pair's landmarks move by
    its back substitution with dc_p = Ad_p dB; bodies R <- cayley(w) R, t <- cayley(w) t + rho, then
    every pair's cameras are recomputed as E_p^-1 B.

    Inertial factors on the body window (``add_keyframe(..., ine=(record, v0))``, ``set_inertial``):
    ``inertial_terms`` with the body poses as the cameras (record in the earlier keyframe's body
    axes, velocities of the body origin, gravity in the body window's world = base_link at frame
    0), added to the combined S and b and eliminated as in the pair window."""

    def __init__(self, K: int, intrs: list, E: list[np.ndarray], params: BAParams):
        from .numpy_rig import inv_rigid, mul4

        self._mul4 = mul4
        self.pairs = [KeyframeWindow(K, intr, params) for intr in intrs]
        self.E = [np.asarray(e, dtype=np.float64) for e in E]
        self.Einv = [inv_rigid(e) for e in self.E]
        self.Ad = [adjoint_rl(ei) for ei in self.Einv]
        self.p = params
        self.B = np.tile(np.eye(4), (params.window, 1, 1))   # body_T_world per slot
        self.ine = np.zeros((params.window, INE_N))
        self.vel = np.zeros((params.window, 3))
        self.bias = np.zeros((params.window, 6))
        self.ine_cfg = (np.zeros(3), np.zeros(3), 0.0, np.zeros(3), 0.0)

    def set_inertial(self, gw: np.ndarray, ba0: np.ndarray, wb: float, bg0: np.ndarray | None = None,
                     wg: float = 0.0) -> None:
        self.ine_cfg = _ine_cfg(gw, ba0, wb, bg0, wg)

    @property
    def frame(self) -> np.ndarray:
        return self.pairs[0].frame

    def order(self) -> list[int]:
        return self.pairs[0].order()

    def cams(self, p: int, B: np.ndarray) -> np.ndarray:
        return np.stack([self._mul4(self.Einv[p], b) for b in B])

    def add_keyframe(self, g: int, B_new: np.ndarray, obs: list[tuple], ine: tuple | None = None) -> int:
        """Keyframe g with body pose ``B_new`` (body_T_world); ``obs[p]`` = (u, v, disp, link) of
        pair p as for ``KeyframeWindow.add_keyframe``; ``ine`` = (record, v0) the body's inertial
        factor from the previous keyframe and its initial velocity."""
        slot = -1
        prev = self.order()[-1] if self.pairs[0].n_kf else -1
        for p, (w, (u, v, disp, link)) in enumerate(zip(self.pairs, obs)):
            slot = w.add_keyframe(g, self._mul4(self.Einv[p], B_new), u, v, disp, link)
        self.B[slot] = B_new
        self.ine[slot] = 0.0 if ine is None else np.asarray(ine[0], dtype=np.float64)
        self.vel[slot] = 0.0 if ine is None else np.asarray(ine[1], dtype=np.float64)
        self.bias[slot] = new_keyframe_bias(self.ine[slot], self.bias, prev)
        return slot

    def solve(self) -> dict:
        p = self.p
        slots = self.order()
        n = len(slots)
        if n < 2:
            return {"n_obs": 0, "n_lm": 0, "pairs": [{"n_obs": 0, "n_lm": 0} for _ in self.pairs]}
        B = self.B[slots].copy()
        obs = [w.prepare(self.cams(q, B)) for q, w in enumerate(self.pairs)]
        for _ in range(p.iters):
            S = p.lam * np.eye(6 * n)
            b = np.zeros(6 * n)
            lins = []
            for q, w in enumerate(self.pairs):
                T = self.cams(q, B)
                lin = w.linearize(obs[q], T[:, :3, :3].copy(), T[:, :3, 3].copy())
                lins.append(lin)
                A = np.kron(np.eye(n), self.Ad[q])
                S = S + A.T @ lin["S"] @ A
                b = b + A.T @ lin["b"]
            ine = inertial_system(self, slots, B[:, :3, :3], B[:, :3, 3], S, b)
            if ine is None:
                dB = np.zeros(6 * n)
                dB[6:] = np.linalg.solve(S[6:, 6:], b[6:])
            else:
                dB = inertial_step(self, slots, S, b, ine)
            dBB = dB.reshape(n, 6)
            for q, w in enumerate(self.pairs):
                dcc = dBB @ self.Ad[q].T                   # dc_p = Ad_p dB per camera
                obs[q]["X"] = obs[q]["X"] + w.landmark_update(obs[q], lins[q], dcc)
            for c in range(1, n):
                ru = cayley(dBB[c, 3:])
                B[c, :3, :3] = ru @ B[c, :3, :3]
                B[c, :3, 3] = ru @ B[c, :3, 3] + dBB[c, :3]
        self.B[slots] = B
        out = {"n_obs": 0, "n_lm": 0, "pairs": []}
        for q, w in enumerate(self.pairs):
            T = self.cams(q, B)
            for c, s in enumerate(slots):
                w.T_cw[s] = T[c]
            r = w._finish(obs[q], T[:, :3, :3], T[:, :3, 3])
            out["pairs"].append(r)
            out["n_obs"] += r["n_obs"]
            out["n_lm"] += r["n_lm"]
        return out


def keyframe_observations(left: dict, K: int):
    """Level-0 (u, v) of every valid keypoint of one image (NaN for padding slots)."""
    kp = left["kp"]
    u, v = level0_coords(kp["x"], kp["y"], kp["level"])
    u = np.where(left["valid"], u, np.nan)
    v = np.where(left["valid"], v, np.nan)
    return u[:K].astype(np.float64), v[:K].astype(np.float64)


def _inv_rigid(T: np.ndarray) -> np.ndarray:
    out = np.eye(4)
    out[:3, :3] = T[:3, :3].T
    out[:3, 3] = -(T[:3, :3].T @ T[:3, 3])
    return out


class BATracker:
    """Drives one pair's ``KeyframeWindow`` from ``OracleTracker.step`` results (in frame order).

    Keyframe g's initial pose composes the previous keyframe's BA estimate with the front end's
    motion since then: ``world_T_cam = W_ba(prev) inv(W_fe(prev)) W_fe(g)`` (front end = the
    tracking chain, ``res['world_T_cam']``), so a BA correction carries forward."""

    def __init__(self, K: int, intr, params: BAParams):
        self.win = KeyframeWindow(K, intr, params)
        self.K = K
        self.p = params
        self.Tfe = np.tile(np.eye(4), (params.window, 1, 1))
        self.temporal: list[np.ndarray] = []   # newest first, the last kf_interval frames
        self.last_solve: dict | None = None

    def step(self, res: dict, imu: tuple | None = None, ine: tuple | None = None) -> dict | None:
        """One frame's tracker result; ``imu`` = (M, w), the keyframe's IMU rotation factor;
        ``ine`` = (record, v0), its inertial factor and initial velocity."""
        g = int(res["frame"])
        cur = res["cur"]
        self.temporal.insert(0, np.asarray(cur["temporal"], dtype=np.int64))
        del self.temporal[self.p.kf_interval:]
        if g % self.p.kf_interval:
            return None
        w = self.win
        W_fe = res["world_T_cam"]
        if w.n_kf == 0:
            T_wc = W_fe.copy()
            link = None
        else:
            prev = w.order()[-1]
            T_wc = _inv_rigid(w.T_cw[prev]) @ _inv_rigid(self.Tfe[prev]) @ W_fe
            link = chain_links(self.temporal[: self.p.kf_interval])
        u, v = keyframe_observations(cur["left"], self.K)
        slot = w.add_keyframe(g, _inv_rigid(T_wc), u, v, np.asarray(cur["disp"], dtype=np.float64), link, imu=imu,
                              ine=ine)
        self.Tfe[slot] = W_fe
        self.last_solve = w.solve()
        return self.last_solve


class RigBATracker:
    """Drives a ``RigKeyframeWindow`` from the pairs' ``OracleTracker.step`` results and the rig's
    body front end (``world_T_body`` of ``RigChain``, world = base_link at frame 0), in frame
    order.  Keyframe g's initial body pose is ``W_ba(prev) inv(W_fe(prev)) W_fe(g)`` in body terms
    (the rig restatement of ``BATracker``)."""

    def __init__(self, K: int, intrs: list, E: list[np.ndarray], params: BAParams):
        self.win = RigKeyframeWindow(K, intrs, E, params)
        self.K = K
        self.p = params
        self.Tfe = np.tile(np.eye(4), (params.window, 1, 1))   # world_T_body at insertion
        self.temporal: list[list[np.ndarray]] = [[] for _ in intrs]
        self.last_solve: dict | None = None

    def step(self, g: int, results: list[dict], world_T_body: np.ndarray, ine: tuple | None = None) -> dict | None:
        for q, res in enumerate(results):
            self.temporal[q].insert(0, np.asarray(res["cur"]["temporal"], dtype=np.int64))
            del self.temporal[q][self.p.kf_interval:]
        if g % self.p.kf_interval:
            return None
        w = self.win
        first = w.pairs[0].n_kf == 0
        if first:
            T_wb = world_T_body.copy()
        else:
            prev = w.order()[-1]
            T_wb = _inv_rigid(w.B[prev]) @ _inv_rigid(self.Tfe[prev]) @ world_T_body
        obs = []
        for q, res in enumerate(results):
            u, v = keyframe_observations(res["cur"]["left"], self.K)
            link = None if first else chain_links(self.temporal[q][: self.p.kf_interval])
            obs.append((u, v, np.asarray(res["cur"]["disp"], dtype=np.float64), link))
        slot = w.add_keyframe(g, _inv_rigid(T_wb), obs, ine=ine)
        self.Tfe[slot] = world_T_body
        self.last_solve = w.solve()
        return self.last_solve
