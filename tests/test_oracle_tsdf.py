"""TSDF oracle (oracle/numpy_tsdf.py) against hand-derived cases: a fronto-parallel wall seen by a
camera at the origin gives sdf = wall - z in front, truncated, nothing behind the band, running
averages with capped weights."""

import numpy as np

from oracle import numpy_tsdf as TS


def test_fronto_parallel_wall():
    H, W = 48, 64
    depth = np.full((H, W), 2000, dtype=np.uint16)          # a wall at 2 m
    origin, dims, s = (-0.1, -0.1, 1.5), (4, 4, 20), 0.05    # z from 1.5 to 2.5 m
    t = np.zeros(dims[::-1], dtype=np.float32)
    w = np.zeros(dims[::-1], dtype=np.float32)
    intr = (50.0, 50.0, (W - 1) / 2, (H - 1) / 2)
    TS.integrate(t, w, depth, np.eye(4), intr, origin, s, 0.2, 10.0, 3.0)
    z = origin[2] + s * (np.arange(dims[2]) + 0.5)
    sdf = 2.0 - z
    band = sdf >= -0.2
    np.testing.assert_array_equal(w[:, 1, 1] > 0, band)
    np.testing.assert_allclose(t[band, 1, 1], np.minimum(sdf[band], 0.2).astype(np.float32), rtol=0, atol=1e-7)
    # three more identical frames: averages unchanged, weights capped at max_weight = 3
    for _ in range(3):
        TS.integrate(t, w, depth, np.eye(4), intr, origin, s, 0.2, 10.0, 3.0)
    assert w.max() == 3.0
    np.testing.assert_allclose(t[band, 1, 1], np.minimum(sdf[band], 0.2), atol=1e-6)
    pts = TS.surface_points(np.transpose(t, (2, 1, 0)).copy(), np.transpose(w, (2, 1, 0)).copy(), (0, 0, 0), 1.0)
    assert pts.shape[1] == 3


def test_zero_depth_and_far_depth_are_ignored():
    depth = np.zeros((10, 10), dtype=np.uint16)
    depth[5, 5] = 12000                                      # 12 m > max_dist
    t = np.zeros((5, 5, 5), dtype=np.float32)
    w = np.zeros((5, 5, 5), dtype=np.float32)
    TS.integrate(t, w, depth, np.eye(4), (5.0, 5.0, 4.5, 4.5), (-0.5, -0.5, 0.5), 0.2, 0.8, 10.0, 100.0)
    assert not w.any()
