"""Constant tables of the detect/describe stages (rows A4-A5 of SURVEY.md §8a).

cuVSLAM's feature front end is closed, so the algorithm is defined here and
restated independently in ``oracle/`` (tests check the two derivations agree byte for byte):

* FAST-9 on the 16-pixel Bresenham circle of radius 3, listed clockwise from 12 o'clock.
* Intensity-centroid orientation on the disc dx^2 + dy^2 <= 15^2, quantised to 30 bins of 12
  degrees with *integer* wedge tests: bin b holds every moment vector v = (m10, m01) with
  cross(u_b, v) >= 0 and cross(u_{b+1}, v) < 0, u_b = round(2^24 (cos, sin)((b - 1/2) * 12 deg)).
* rBRIEF-256: 256 point pairs drawn once from a seeded N(0, 6.2^2) (numpy PCG64, seed 0xB1EF),
  rounded and clipped to [-13, 13]; the pattern is pre-rotated to each bin centre b * 12 deg
  and rounded (floor(x + 1/2)), so the device only does table lookups.
"""

from __future__ import annotations

import numpy as np

FAST_CIRCLE = np.array(
    [(0, -3), (1, -3), (2, -2), (3, -1), (3, 0), (3, 1), (2, 2), (1, 3),
     (0, 3), (-1, 3), (-2, 2), (-3, 1), (-3, 0), (-3, -1), (-2, -2), (-1, -3)],
    dtype=np.int32,
)
ORIENT_RADIUS = 15
N_ANGLE_BINS = 30
BRIEF_BITS = 256
BRIEF_SEED = 0xB1EF
BRIEF_SIGMA = 31.0 / 5.0
BRIEF_CLIP = 13
WEDGE_SCALE_BITS = 24


def _round_half_up(x: np.ndarray) -> np.ndarray:
    return np.floor(x + 0.5)


def brief_pattern() -> np.ndarray:
    """(256, 4) int32 rows (px, py, qx, qy) of the unrotated pattern."""
    rng = np.random.default_rng(BRIEF_SEED)
    pts = _round_half_up(rng.normal(0.0, BRIEF_SIGMA, size=(BRIEF_BITS, 4)))
    pts = np.clip(pts, -BRIEF_CLIP, BRIEF_CLIP).astype(np.int32)
    same = (pts[:, 0] == pts[:, 2]) & (pts[:, 1] == pts[:, 3])
    pts[same, 2] = np.where(pts[same, 2] < BRIEF_CLIP, pts[same, 2] + 1, pts[same, 2] - 1)
    return pts


def rotated_brief_table() -> np.ndarray:
    """(30, 256, 4) int8: the pattern rotated to each orientation-bin centre."""
    pat = brief_pattern().astype(np.float64)
    out = np.empty((N_ANGLE_BINS, BRIEF_BITS, 4), dtype=np.int8)
    for b in range(N_ANGLE_BINS):
        th = 2.0 * np.pi * b / N_ANGLE_BINS
        c, s = np.cos(th), np.sin(th)
        for k in (0, 2):
            x, y = pat[:, k], pat[:, k + 1]
            out[b, :, k] = _round_half_up(c * x - s * y)
            out[b, :, k + 1] = _round_half_up(s * x + c * y)
    return out


def wedge_table() -> np.ndarray:
    """(31, 2) int64 fixed-point boundary directions u_0..u_30 (u_30 == u_0)."""
    b = np.arange(N_ANGLE_BINS + 1, dtype=np.float64)
    beta = (b - 0.5) * (2.0 * np.pi / N_ANGLE_BINS)
    scale = float(1 << WEDGE_SCALE_BITS)
    tab = np.stack([_round_half_up(np.cos(beta) * scale), _round_half_up(np.sin(beta) * scale)], axis=1)
    tab[N_ANGLE_BINS] = tab[0]
    return tab.astype(np.int64)


def orient_disc() -> np.ndarray:
    """(N, 2) int32 offsets (dx, dy) of the orientation disc, row-major order."""
    r = ORIENT_RADIUS
    dy, dx = np.mgrid[-r : r + 1, -r : r + 1]
    m = dx * dx + dy * dy <= r * r
    return np.stack([dx[m], dy[m]], axis=1).astype(np.int32)


def orient_half_widths() -> np.ndarray:
    """(16,) int32 umax[|dy|] = max dx with dx^2 + dy^2 <= 15^2 (device-side disc description)."""
    r = ORIENT_RADIUS
    return np.array([int(np.floor(np.sqrt(r * r - d * d) + 1e-9)) for d in range(r + 1)], dtype=np.int32)
