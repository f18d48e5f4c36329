"""SURVEY.md §8f item 4 — RGB-D dense mapping (nvblox-shaped TSDF integration), CPU restatement.

TEST INFRASTRUCTURE (see ``oracle/__init__.py``): the checker for ``k_tsdf.hip``, never imported
by the product.  The reference runs nvblox (``launch/thor_nvblox.launch.py:26-36``: voxel 0.05 m,
truncation 4 voxels, max integration distance 10 m) on the RGB + u16-depth topics of
``scripts/run_pipeline.py:218-256``; nvblox is an external package absent from
``/root/reference``, so this file restates its projective TSDF integrator and is the spec here
(parity against nvblox itself is unpinned).

Volume: a dense grid of ``dims = (nx, ny, nz)`` voxels of size ``s`` whose corner is ``origin``
(metres, in the tracking world = rectified left camera at frame 0, RDF); voxel (i, j, k) has centre
origin + s (i + 1/2, j + 1/2, k + 1/2) and stores a truncated signed distance (f32, metres) and a
weight (f32); storage order [k][j][i].

Integration of one depth frame (u16 mm, aligned to the colour camera, undistorted through the same
table as the tracking image) with camera pose cam_T_world, per voxel, in f64:

    p = R c + t                                     (c: voxel centre; row-wise sums, fixed order)
    skip unless p_z > 0
    u = fx p_x / p_z + cx, v = fy p_y / p_z + cy;  ix = floor(u + 1/2), iy = floor(v + 1/2)
    skip unless 0 <= ix < W and 0 <= iy < H
    (ix, iy) <- the raw pixel of the undistortion table (as A6's RGB-D depth lookup)
    d = mm * 0.001;  skip unless 0 < d <= max_dist
    sdf = d - p_z;   skip if sdf < -trunc
    obs = min(sdf, trunc)
    w' = w + 1;  tsdf' = (tsdf * w + obs) / w';  w' = min(w', max_weight)     (stored as f32)

Frames are integrated in order; a batch of frames gives the same result as one call per frame.

Colour layer (nvblox's colour integration on the RGB image aligned with the depth): with a BGR
image, every voxel the frame updates whose surface distance is inside the truncation band
(|sdf| <= trunc) also averages the colour of the same (undistorted) pixel, R, G, B in [0, 255]:
cw' = cw + 1;  c' = (c * cw + obs) / cw' per channel;  cw' = min(cw', max_weight)  (stored as f32).
"""

from __future__ import annotations

import numpy as np

RECT_BITS = 5


def voxel_centres(origin, dims, s) -> np.ndarray:
    nx, ny, nz = dims
    k, j, i = np.meshgrid(np.arange(nz), np.arange(ny), np.arange(nx), indexing="ij")
    return np.stack([origin[0] + s * (i + 0.5), origin[1] + s * (j + 0.5), origin[2] + s * (k + 0.5)], axis=-1)


def integrate(tsdf: np.ndarray, weight: np.ndarray, depth_mm: np.ndarray, cam_T_world: np.ndarray, intr,
              origin, s: float, trunc: float, max_dist: float, max_weight: float, mp: np.ndarray | None = None,
              bgr: np.ndarray | None = None, color: np.ndarray | None = None, color_w: np.ndarray | None = None):
    """One frame into (tsdf, weight) [nz][ny][nx] f32, in place; with ``bgr`` [H][W][3] u8 also the
    colour layer ``color`` [nz][ny][nx][3] (R, G, B) f32 and ``color_w`` f32."""
    fx, fy, cx, cy = intr
    h, w = depth_mm.shape
    c = voxel_centres(origin, tsdf.shape[::-1], s)
    R, t = cam_T_world[:3, :3], cam_T_world[:3, 3]
    px = ((R[0, 0] * c[..., 0] + R[0, 1] * c[..., 1]) + R[0, 2] * c[..., 2]) + t[0]
    py = ((R[1, 0] * c[..., 0] + R[1, 1] * c[..., 1]) + R[1, 2] * c[..., 2]) + t[1]
    pz = ((R[2, 0] * c[..., 0] + R[2, 1] * c[..., 1]) + R[2, 2] * c[..., 2]) + t[2]
    ok = pz > 0.0
    zs = np.where(ok, pz, 1.0)
    u = fx * px / zs + cx
    v = fy * py / zs + cy
    ix = np.floor(u + 0.5)
    iy = np.floor(v + 0.5)
    ok &= (ix >= 0) & (ix < w) & (iy >= 0) & (iy < h)
    ix = np.where(ok, ix, 0).astype(np.int64)
    iy = np.where(ok, iy, 0).astype(np.int64)
    if mp is not None:
        m = mp[iy, ix].astype(np.int64)
        ix = np.clip((m[..., 0] + 16) >> RECT_BITS, 0, w - 1)
        iy = np.clip((m[..., 1] + 16) >> RECT_BITS, 0, h - 1)
    d = depth_mm[iy, ix].astype(np.float64) * 0.001
    ok &= (d > 0.0) & (d <= max_dist)
    sdf = d - pz
    ok &= sdf >= -trunc
    obs = np.minimum(sdf, trunc)
    w0 = weight.astype(np.float64)
    w1 = w0 + 1.0
    new = (tsdf.astype(np.float64) * w0 + obs) / w1
    tsdf[ok] = new[ok].astype(np.float32)
    weight[ok] = np.minimum(w1, max_weight)[ok].astype(np.float32)
    if bgr is not None:
        band = ok & (sdf <= trunc)
        obs_c = bgr[iy, ix][..., ::-1].astype(np.float64)              # R, G, B of the same pixel
        cw0 = color_w.astype(np.float64)
        cw1 = cw0 + 1.0
        newc = (color.astype(np.float64) * cw0[..., None] + obs_c) / cw1[..., None]
        color[band] = newc[band].astype(np.float32)
        color_w[band] = np.minimum(cw1, max_weight)[band].astype(np.float32)


def surface_points(tsdf: np.ndarray, weight: np.ndarray, origin, s: float) -> np.ndarray:
    """Voxel centres next to a zero crossing along x (observed on both sides): a crude surface sample."""
    a, b = tsdf[:, :, :-1], tsdf[:, :, 1:]
    obs = (weight[:, :, :-1] > 0) & (weight[:, :, 1:] > 0)
    k, j, i = np.nonzero(obs & (a > 0) & (b <= 0))
    return np.stack([origin[0] + s * (i + 0.5), origin[1] + s * (j + 0.5), origin[2] + s * (k + 0.5)], axis=1)
