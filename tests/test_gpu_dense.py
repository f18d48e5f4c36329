"""Dense-map outputs on the GPU (k_dense.hip) vs oracle/numpy_dense.py: marching-cubes triangles,
ESDF and the 2-D distance slice bit-exact (f32 bits, NaN included) on a sphere volume, on random
sign volumes with unobserved voxels (every ambiguous face configuration), on a volume integrated
from rendered RGB-D frames with the device-tracked poses, and at the edges (no observed voxel, a
one-voxel-thick volume, R = 0, the triangle buffer grown on a larger volume)."""

from __future__ import annotations

import numpy as np
import pytest

from oracle import numpy_dense as D
from thor_slam_amd.calib import extract_cameras, stereo_pairs, stereo_rectify
from thor_slam_amd.camera.rig import CameraRig
from thor_slam_amd.params import HipSlamConfig
from thor_slam_amd.synthetic import SyntheticStereoSource

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def handle():
    from thor_slam_amd._lib import Handle

    src = SyntheticStereoSource(seed=3, n_frames=2)
    cams = extract_cameras(CameraRig([src]).calibration, 2)
    (li, ri), = stereo_pairs(cams)
    h = Handle([stereo_rectify(cams[li], cams[ri])], HipSlamConfig(), max_batch=2)
    yield h
    h.close()


def _bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)


def _check_volume(h, t, w, origin, s, max_dists=(0.5, 2.0), band=None):
    nz, ny, nx = t.shape
    h.tsdf_init(origin, (nx, ny, nz), s)
    h.tsdf_write(t, w)
    got = h.mesh()
    want = D.extract_mesh(t, w, origin, s, 1e-4)
    assert got.shape == want.shape
    np.testing.assert_array_equal(_bits(got), _bits(want))
    for md in max_dists:
        np.testing.assert_array_equal(_bits(h.esdf(md)), _bits(D.esdf(t, w, s, md)))
    y0, y1 = band if band else (ny // 3, max(ny // 3 + 1, 2 * ny // 3))
    np.testing.assert_array_equal(_bits(h.esdf_slice(y0, y1, 1.0)), _bits(D.esdf_slice(t, w, s, 1.0, y0, y1)))
    return got


def test_sphere(handle):
    n, s, origin = 40, 0.05, (-1.0, -1.0, -1.0)
    ax = origin[0] + s * (np.arange(n) + 0.5)
    Z, Y, X = np.meshgrid(ax, ax, ax, indexing="ij")
    t = np.clip(np.sqrt(X ** 2 + Y ** 2 + Z ** 2) - 0.6, -0.2, 0.2).astype(np.float32)
    m = _check_volume(handle, t, np.ones_like(t), origin, s)
    assert m.shape[0] > 5000


@pytest.mark.parametrize("seed", [0, 1])
def test_random_signs_and_unobserved(handle, seed):
    rng = np.random.default_rng(seed)
    t = rng.uniform(-0.3, 0.3, (17, 23, 29)).astype(np.float32)
    w = rng.choice(np.array([0.0, 1.0, 3.0], dtype=np.float32), size=t.shape, p=[0.1, 0.6, 0.3])
    m = _check_volume(handle, t, w, (0.25, -1.0, 2.0), 0.1, max_dists=(0.1, 0.35, 3.0, 8.0))   # R = 1, 3, 30 (LDS passes), 80 (direct)
    assert m.shape[0] > 10000


def test_mesh_vertex_colours():
    """With the colour layer every vertex takes its edge's nearer voxel's colour (oracle bits)."""
    from thor_slam_amd._lib import Handle

    src = SyntheticStereoSource(seed=3, n_frames=2)
    cams = extract_cameras(CameraRig([src]).calibration, 2)
    (li, ri), = stereo_pairs(cams)
    h = Handle([stereo_rectify(cams[li], cams[ri])], HipSlamConfig(), max_batch=2)
    rng = np.random.default_rng(5)
    t = rng.uniform(-0.3, 0.3, (13, 17, 19)).astype(np.float32)
    w = rng.choice(np.array([0.0, 1.0, 2.0], dtype=np.float32), size=t.shape, p=[0.1, 0.6, 0.3])
    col = rng.uniform(0, 255, t.shape + (3,)).astype(np.float32)
    h.tsdf_color(True)
    h.tsdf_init((0.0, 0.5, 1.0), (19, 17, 13), 0.1)
    h.tsdf_write(t, w)
    h.tsdf_write_color(col, np.ones_like(w))
    tris, cols = h.mesh(colors=True)
    want_t, want_c = D.extract_mesh(t, w, (0.0, 0.5, 1.0), 0.1, 1e-4, color=col)
    assert tris.shape[0] > 1000
    np.testing.assert_array_equal(_bits(tris), _bits(want_t))
    np.testing.assert_array_equal(_bits(cols), _bits(want_c))
    h.close()


def test_edges(handle):
    t = np.full((6, 5, 4), 0.1, dtype=np.float32)
    w = np.zeros_like(t)
    _check_volume(handle, t, w, (0, 0, 0), 0.1, max_dists=(0.05, 1.0))          # nothing observed: R = 0 too
    assert handle.mesh().shape == (0, 3, 3) and np.isnan(handle.esdf()).all()
    t1 = np.random.default_rng(2).uniform(-1, 1, (7, 1, 9)).astype(np.float32)
    _check_volume(handle, t1, np.ones_like(t1), (0, 0, 0), 0.2, band=(0, 1))      # one voxel thick: no cubes
    assert handle.mesh().shape == (0, 3, 3)
    small = np.random.default_rng(3).uniform(-1, 1, (4, 4, 4)).astype(np.float32)
    _check_volume(handle, small, np.ones_like(small), (0, 0, 0), 0.2)
    big = np.random.default_rng(4).uniform(-1, 1, (30, 30, 30)).astype(np.float32)
    _check_volume(handle, big, np.ones_like(big), (0, 0, 0), 0.2)                # triangle buffer grows


def test_integrated_volume_end_to_end():
    """A TSDF integrated from rendered RGB-D frames with the device-tracked poses, then meshed."""
    import torch

    from thor_slam_amd._lib import Handle
    from thor_slam_amd.calib import rgbd_pairs, rgbd_undistort
    from thor_slam_amd.synthetic import SyntheticRGBDSource

    W, H, n = 320, 240, 6
    src = SyntheticRGBDSource(width=W, height=H)
    cams = extract_cameras(CameraRig([src]).calibration, 2)
    (ci, _), = rgbd_pairs(cams)
    rect = rgbd_undistort(cams[ci])
    h = Handle([rect], HipSlamConfig(rgbd=True, n_features=1000, n_levels=3), max_batch=n)
    rec = src.render_rgbd_sequence(n)[:, None, :]
    dev = torch.from_numpy(np.ascontiguousarray(rec)).cuda()
    h.submit(dev.data_ptr(), n, torch.cuda.current_stream().cuda_stream)
    h.read_poses(n)
    origin, dims, s = (-2.0, -1.5, 0.5), (80, 60, 100), 0.05
    h.tsdf_init(origin, dims, s, 4.0, 10.0, 100.0)
    h.tsdf_integrate(dev.data_ptr() + 3 * W * H, 5 * W * H, n)
    t, w = h.tsdf_read()
    assert (w > 0).sum() > 10000
    got = h.mesh()
    want = D.extract_mesh(t, w, origin, s, 1e-4)
    assert got.shape[0] > 1000
    np.testing.assert_array_equal(_bits(got), _bits(want))
    np.testing.assert_array_equal(_bits(h.esdf(2.0)), _bits(D.esdf(t, w, s, 2.0)))
    np.testing.assert_array_equal(_bits(h.esdf_slice(20, 40, 2.0)), _bits(D.esdf_slice(t, w, s, 2.0, 20, 40)))
    h.close()
