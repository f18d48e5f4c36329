"""Calibration semantics at the boundary (row A1/A2 of SURVEY.md §8a) — host side, run once.

Restates the behaviour of the component this back end replaces, ``IsaacRosAdapter``
(``thor_slam/slam/adapters/isaac_ros.py``):

* global camera order            ``_extract_cameras``  isaac_ros.py:138-157
* distortion-model selection     isaac_ros.py:370-383 (>=8 coeffs -> rational_polynomial[:8], 5 ->
  plumb_bob, 4 -> equidistant, otherwise zero-padded plumb_bob)
* stereo baseline / projection   isaac_ros.py:387-408 (t_lr = R_l^T (t_r - t_l), P[0,3] = -fx t_lr[0])
* confidence from covariance     isaac_ros.py:312     (clamp(1 / (1 + tr(cov[:3,:3])), 0, 1))

and builds what cuVSLAM computes internally when ``rectified_images:=false`` (Makefile:80): a
Bouguet-style stereo rectification (half-rotation of each camera + a common rotation that aligns
the baseline with +x) and per-camera remap tables in 1/32-pixel fixed point
(``RECT_FRAC_BITS``).  The tables are what the ``rectify_pyramid`` kernel consumes.
"""

from __future__ import annotations

from dataclasses import dataclass

import numpy as np
from scipy.spatial.transform import Rotation

from .camera.rig import RigCalibration
from .camera.types import Extrinsics, Intrinsics
from .slam.interface import CameraConfig

RECT_FRAC_BITS = 5
RECT_ONE = 1 << RECT_FRAC_BITS

# Reference isaac_ros.py:42-49 — RDF optical axes expressed in FLU base axes.
RDF_TO_FLU_MATRIX = np.array([[0, 0, 1, 0], [-1, 0, 0, 0], [0, -1, 0, 0], [0, 0, 0, 1]], dtype=np.float64)


def extract_cameras(cal: RigCalibration, num_cameras: int) -> list[CameraConfig]:
    """Flat camera list: sorted source names x cam_idx, capped at ``num_cameras``."""
    cams: list[CameraConfig] = []
    for source in sorted(cal.intrinsics.keys()):
        intr_list = cal.intrinsics[source]
        extr_list = cal.get_world_extrinsics(source) or cal.extrinsics.get(source, [])
        for cam_idx, intr in enumerate(intr_list):
            if len(cams) >= num_cameras:
                break
            extr = extr_list[cam_idx] if cam_idx < len(extr_list) else Extrinsics(np.eye(3), np.zeros(3))
            cams.append(CameraConfig(intr, extr, source, cam_idx))
    return cams


def stereo_pairs(cams: list[CameraConfig]) -> list[tuple[int, int]]:
    """(left, right) global indices: a cam_idx=1 camera directly after cam_idx=0 of its source."""
    pairs = []
    for i, cam in enumerate(cams):
        if cam.cam_idx == 1 and i > 0 and cams[i - 1].source_name == cam.source_name and cams[i - 1].cam_idx == 0:
            pairs.append((i - 1, i))
    return pairs


def distortion_model(coeffs: np.ndarray) -> tuple[str, list[float]]:
    d = np.asarray(coeffs, dtype=np.float64).flatten().tolist()
    if len(d) >= 8:
        return "rational_polynomial", d[:8]
    if len(d) == 5:
        return "plumb_bob", d
    if len(d) == 4:
        return "equidistant", d
    return "plumb_bob", (d + [0.0] * 5)[:5]


def stereo_projection(left: CameraConfig, right: CameraConfig) -> tuple[np.ndarray, float]:
    """The right camera's ROS projection matrix P (3x4) and the baseline t_lr[0] [m]."""
    t_lr = left.extrinsics.rotation.T @ (np.asarray(right.extrinsics.translation) - np.asarray(left.extrinsics.translation))
    baseline = float(t_lr[0])
    p = np.zeros((3, 4))
    p[:3, :3] = right.intrinsics.matrix
    p[0, 3] = -float(right.intrinsics.matrix[0, 0]) * baseline
    return p, baseline


def confidence_from_covariance(cov: np.ndarray | None) -> float:
    if cov is None:
        return 1.0
    return float(max(0.0, min(1.0, 1.0 / (1.0 + np.trace(np.asarray(cov)[:3, :3])))))


# --------------------------------------------------------------------------------------
# distortion models (normalised coordinates)
# --------------------------------------------------------------------------------------
def distort_normalized(x: np.ndarray, y: np.ndarray, coeffs: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
    """Apply the selected distortion model to undistorted normalised coordinates."""
    model, d = distortion_model(coeffs)
    if model == "equidistant":
        k1, k2, k3, k4 = d
        r = np.sqrt(x * x + y * y)
        th = np.arctan(r)
        th2 = th * th
        thd = th * (1 + th2 * (k1 + th2 * (k2 + th2 * (k3 + th2 * k4))))
        scale = np.where(r > 1e-12, thd / np.where(r > 1e-12, r, 1.0), 1.0)
        return x * scale, y * scale
    k = list(d) + [0.0] * (8 - len(d))
    k1, k2, p1, p2, k3, k4, k5, k6 = k[:8]
    r2 = x * x + y * y
    radial = (1 + r2 * (k1 + r2 * (k2 + r2 * k3))) / (1 + r2 * (k4 + r2 * (k5 + r2 * k6)))
    xd = x * radial + 2 * p1 * x * y + p2 * (r2 + 2 * x * x)
    yd = y * radial + p1 * (r2 + 2 * y * y) + 2 * p2 * x * y
    return xd, yd


def undistort_normalized(xd: np.ndarray, yd: np.ndarray, coeffs: np.ndarray, iters: int = 20) -> tuple[np.ndarray, np.ndarray]:
    """Fixed-point iteration inverse of ``distort_normalized`` (used by the synthetic renderer)."""
    x, y = xd.copy(), yd.copy()
    for _ in range(iters):
        dx, dy = distort_normalized(x, y, coeffs)
        x = x - (dx - xd)
        y = y - (dy - yd)
    return x, y


# --------------------------------------------------------------------------------------
# stereo rectification
# --------------------------------------------------------------------------------------
@dataclass
class StereoRectification:
    width: int
    height: int
    fx: float
    fy: float
    cx: float
    cy: float
    baseline: float            # metres, > 0 when the right camera sits at +x of the left
    rect_left: np.ndarray      # 3x3: rectified_left <- left optical
    rect_right: np.ndarray     # 3x3: rectified_right <- right optical
    map_left: np.ndarray       # (H, W, 2) int32, source (x, y) * 32 for every rectified pixel
    map_right: np.ndarray
    is_identity: bool

    def left_optical_T_rect(self) -> np.ndarray:
        m = np.eye(4)
        m[:3, :3] = self.rect_left.T
        return m


def _rodrigues(v: np.ndarray) -> np.ndarray:
    return Rotation.from_rotvec(np.asarray(v, dtype=np.float64)).as_matrix()


def rectify_map(intr: Intrinsics, rect_rot: np.ndarray, fx: float, fy: float, cx: float, cy: float) -> np.ndarray:
    """Fixed-point remap table: rectified pixel -> raw pixel of this camera."""
    w, h = intr.width, intr.height
    v, u = np.mgrid[0:h, 0:w].astype(np.float64)
    ray = np.stack([(u - cx) / fx, (v - cy) / fy, np.ones_like(u)], axis=-1) @ rect_rot  # R^T applied
    xn = ray[..., 0] / ray[..., 2]
    yn = ray[..., 1] / ray[..., 2]
    xd, yd = distort_normalized(xn, yn, intr.coeffs)
    k = np.asarray(intr.matrix, dtype=np.float64)
    su = k[0, 0] * xd + k[0, 1] * yd + k[0, 2]
    sv = k[1, 1] * yd + k[1, 2]
    lim_x, lim_y = (w + 1) * RECT_ONE, (h + 1) * RECT_ONE
    mx = np.clip(np.floor(su * RECT_ONE + 0.5), -2 * RECT_ONE, lim_x).astype(np.int32)
    my = np.clip(np.floor(sv * RECT_ONE + 0.5), -2 * RECT_ONE, lim_y).astype(np.int32)
    return np.stack([mx, my], axis=-1)


def stereo_rectify(left: CameraConfig, right: CameraConfig) -> StereoRectification:
    """Bouguet rectification of a stereo pair from intrinsics + (world) extrinsics.

    x_r = R x_l + T with R, T from the relative pose; each camera is rotated by half of R, then a
    common rotation aligns the baseline with the x axis.  The rectified pair shares
    f = min(focal lengths) and the mean principal point (zero-disparity convention).
    """
    wl = left.extrinsics.to_4x4_matrix()
    wr = right.extrinsics.to_4x4_matrix()
    l_T_r = np.linalg.inv(wl) @ wr
    r_T_l = np.linalg.inv(l_T_r)
    rot, trans = r_T_l[:3, :3], r_T_l[:3, 3]

    om = Rotation.from_matrix(rot).as_rotvec()
    r_r = _rodrigues(-0.5 * om)
    t = r_r @ trans
    idx = 0 if abs(t[0]) > abs(t[1]) else 1
    uu = np.zeros(3)
    uu[idx] = 1.0 if t[idx] > 0 else -1.0
    ww = np.cross(t, uu)
    nw = np.linalg.norm(ww)
    if nw > 0.0:
        ww = ww * (np.arccos(min(1.0, abs(t[idx]) / np.linalg.norm(t))) / nw)
    w_r = _rodrigues(ww)
    rect_l = w_r @ r_r.T
    rect_r = w_r @ r_r
    t_new = rect_r @ trans

    kl = np.asarray(left.intrinsics.matrix, dtype=np.float64)
    kr = np.asarray(right.intrinsics.matrix, dtype=np.float64)
    f = float(min(kl[0, 0], kl[1, 1], kr[0, 0], kr[1, 1]))
    cx = float(0.5 * (kl[0, 2] + kr[0, 2]))
    cy = float(0.5 * (kl[1, 2] + kr[1, 2]))
    if (left.intrinsics.width, left.intrinsics.height) != (right.intrinsics.width, right.intrinsics.height):
        raise ValueError("stereo pair cameras must share the image size")
    map_l = rectify_map(left.intrinsics, rect_l, f, f, cx, cy)
    map_r = rectify_map(right.intrinsics, rect_r, f, f, cx, cy)
    h, w = map_l.shape[:2]
    ident = np.stack(np.meshgrid(np.arange(w), np.arange(h)), axis=-1).astype(np.int32) * RECT_ONE
    is_identity = bool(np.array_equal(map_l, ident) and np.array_equal(map_r, ident))
    return StereoRectification(
        width=w,
        height=h,
        fx=f,
        fy=f,
        cx=cx,
        cy=cy,
        baseline=float(-t_new[0]),
        rect_left=rect_l,
        rect_right=rect_r,
        map_left=map_l,
        map_right=map_r,
        is_identity=is_identity,
    )


def rgbd_pairs(cams: list[CameraConfig]) -> list[tuple[int, int]]:
    """(colour, depth) global indices of RGB-D sources: cam_idx 0 = the colour camera (BGR),
    cam_idx 1 = the depth image aligned to it (``get_latest_rgbd_frames`` order, luxonis.py:876-919)."""
    return stereo_pairs(cams)


def rgbd_undistort(color: CameraConfig) -> StereoRectification:
    """Undistortion of a colour camera whose depth image is aligned to it (same K and D,
    luxonis.py:1018-1030): pinhole f = min(fx, fy) at the camera's principal point, no rotation.
    The depth is sampled through the same table (nearest raw pixel).  ``baseline`` is the virtual
    1 m the device uses to store depth as disparity fx / Z."""
    k = np.asarray(color.intrinsics.matrix, dtype=np.float64)
    f = float(min(k[0, 0], k[1, 1]))
    cx, cy = float(k[0, 2]), float(k[1, 2])
    mp = rectify_map(color.intrinsics, np.eye(3), f, f, cx, cy)
    h, w = mp.shape[:2]
    ident = np.stack(np.meshgrid(np.arange(w), np.arange(h)), axis=-1).astype(np.int32) * RECT_ONE
    return StereoRectification(width=w, height=h, fx=f, fy=f, cx=cx, cy=cy, baseline=1.0, rect_left=np.eye(3),
                               rect_right=np.eye(3), map_left=mp, map_right=mp, is_identity=bool(np.array_equal(mp, ident)))
