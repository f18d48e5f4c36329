"""RGB-D dense mapping: ``k_tsdf.hip`` vs ``oracle/numpy_tsdf.py`` on
identical depth frames and poses — TSDF and weight volumes bit-exact (same IEEE f64 operations,
f32 storage after every frame), for host poses and for the device-resident tracked poses, with and
without an undistortion table; a batch equals one call per frame; the integrated surface sits at
the rendered depth."""

from __future__ import annotations

import numpy as np
import pytest

from helpers import DISTORTION
from oracle import numpy_tsdf as TS
from thor_slam_amd.calib import extract_cameras, rgbd_pairs, rgbd_undistort
from thor_slam_amd.camera.rig import CameraRig
from thor_slam_amd.params import HipSlamConfig
from thor_slam_amd.synthetic import SyntheticRGBDSource

pytestmark = pytest.mark.gpu

ORIGIN = (-2.0, -1.5, 0.5)     # rect world (frame-0 camera, RDF): 4 m x 3 m x 5 m ahead of it
DIMS = (80, 60, 100)
VOX, TRUNC_VOX, MAX_D, MAX_W = 0.05, 4.0, 10.0, 100.0


def _inv(T):
    """cam_T_world with k_tsdf_poses' expression order."""
    out = np.eye(4)
    for r in range(3):
        for k in range(3):
            out[r, k] = T[k, r]
        out[r, 3] = -((T[0, r] * T[0, 3] + T[1, r] * T[1, 3]) + T[2, r] * T[2, 3])
    return out


def _setup(distorted: bool, n: int, width=320, height=240):
    import torch

    from thor_slam_amd._lib import Handle

    src = SyntheticRGBDSource(width=width, height=height, distortion=DISTORTION if distorted else None)
    cams = extract_cameras(CameraRig([src]).calibration, 2)
    (ci, _), = rgbd_pairs(cams)
    rect = rgbd_undistort(cams[ci])
    cfg = HipSlamConfig(rgbd=True, n_features=1000, n_levels=3)
    rec = src.render_rgbd_sequence(n)[:, None, :]
    h = Handle([rect], cfg, max_batch=n)
    dev = torch.from_numpy(np.ascontiguousarray(rec)).cuda()
    h.submit(dev.data_ptr(), n, torch.cuda.current_stream().cuda_stream)
    res = h.read_poses(n)
    depth = [rec[f, 0, 3 * width * height:].view(np.uint16).reshape(height, width) for f in range(n)]
    return src, rect, h, dev, res, depth


def _oracle(rect, depth, world_T_cam, use, bgr=None):
    t = np.zeros(DIMS[::-1], dtype=np.float32)
    w = np.zeros(DIMS[::-1], dtype=np.float32)
    col = np.zeros(DIMS[::-1] + (3,), dtype=np.float32)
    cw = np.zeros(DIMS[::-1], dtype=np.float32)
    intr = (rect.fx, rect.fy, rect.cx, rect.cy)
    for f, (d, T, u) in enumerate(zip(depth, world_T_cam, use)):
        if u:
            TS.integrate(t, w, d, _inv(T), intr, ORIGIN, VOX, TRUNC_VOX * VOX, MAX_D, MAX_W,
                         None if rect.is_identity else rect.map_left,
                         bgr=None if bgr is None else bgr[f], color=col, color_w=cw)
    return (t, w) if bgr is None else (t, w, col, cw)


@pytest.mark.parametrize("distorted", [False, True])
def test_tsdf_host_poses_bit_exact(distorted):
    n = 4
    src, rect, h, dev, res, depth = _setup(distorted, n)
    W, H = rect.width, rect.height
    poses = res["T_abs"][:, 0]
    h.tsdf_init(ORIGIN, DIMS, VOX, TRUNC_VOX, MAX_D, MAX_W)
    h.tsdf_integrate(dev.data_ptr() + 3 * W * H, 5 * W * H, n, world_T_cam=poses)
    t, w = h.tsdf_read()
    want_t, want_w = _oracle(rect, depth, poses, [True] * n)
    assert (want_w > 0).sum() > 10000
    np.testing.assert_array_equal(w, want_w)
    np.testing.assert_array_equal(t, want_t)
    h.close()


def test_tsdf_device_poses_and_batch_equivalence():
    n = 4
    src, rect, h, dev, res, depth = _setup(False, n)
    W, H = rect.width, rect.height
    h.tsdf_init(ORIGIN, DIMS, VOX, TRUNC_VOX, MAX_D, MAX_W)
    h.tsdf_integrate(dev.data_ptr() + 3 * W * H, 5 * W * H, n, first_frame=0)   # device-resident poses
    t_dev, w_dev = h.tsdf_read()
    st = res["stats"][:, 0, 0]
    want_t, want_w = _oracle(rect, depth, res["T_abs"][:, 0], [s == 0 or (s == 2 and f == 0) for f, s in enumerate(st)])
    np.testing.assert_array_equal(w_dev, want_w)
    np.testing.assert_array_equal(t_dev, want_t)
    # one frame per call == the whole batch in one launch; a NaN pose skips its frame
    h.reset()
    h.tsdf_init(ORIGIN, DIMS, VOX, TRUNC_VOX, MAX_D, MAX_W)
    for f in range(n):
        h.tsdf_integrate(dev[f:].data_ptr() + 3 * W * H, 5 * W * H, 1, world_T_cam=res["T_abs"][f:f + 1, 0])
    nan = np.full((1, 4, 4), np.nan)
    h.tsdf_integrate(dev.data_ptr() + 3 * W * H, 5 * W * H, 1, world_T_cam=nan)
    t1, w1 = h.tsdf_read()
    np.testing.assert_array_equal(w1, want_w)
    np.testing.assert_array_equal(t1, want_t)
    h.close()


def test_tsdf_surface_at_rendered_depth():
    src, rect, h, dev, res, depth = _setup(False, 1)
    W, H = rect.width, rect.height
    h.tsdf_init(ORIGIN, DIMS, VOX, TRUNC_VOX, MAX_D, MAX_W)
    h.tsdf_integrate(dev.data_ptr() + 3 * W * H, 5 * W * H, 1, world_T_cam=np.eye(4)[None])
    t, w = h.tsdf_read()
    h.close()
    # the voxel column on the optical axis (x = y = 0): the zero crossing is at the centre depth
    i = int((0.0 - ORIGIN[0]) / VOX)
    j = int((0.0 - ORIGIN[1]) / VOX)
    col_t, col_w = t[:, j, i], w[:, j, i]
    ks = np.nonzero((col_w[:-1] > 0) & (col_w[1:] > 0) & (col_t[:-1] > 0) & (col_t[1:] <= 0))[0]
    assert ks.size == 1
    k = ks[0]
    z0, z1 = ORIGIN[2] + VOX * (k + 0.5), ORIGIN[2] + VOX * (k + 1.5)
    zc = z0 + (z1 - z0) * col_t[k] / (col_t[k] - col_t[k + 1])
    d = depth[0][int(rect.cy + 0.5), int(rect.cx + 0.5)] * 0.001
    assert abs(zc - d) < 0.03, (zc, d)


def test_tsdf_brick_cull_wide_volume():
    """A volume all around the camera (behind it, beside it, beyond the integration distance) and
    rotated poses: the per-brick frustum cull must never drop an update the per-voxel test makes
    (odd dims exercise partial bricks at every border)."""
    n = 4
    src, rect, h, dev, res, depth = _setup(True, n)
    W, H = rect.width, rect.height
    origin, dims = (-3.1, -1.9, -2.3), (123, 77, 141)
    rng = np.random.default_rng(7)
    poses = []
    for f in range(n):
        a = rng.normal(size=3) * 0.4
        K = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
        th = np.linalg.norm(a)
        R = np.eye(3) + np.sin(th) / th * K + (1 - np.cos(th)) / th ** 2 * K @ K
        T = np.eye(4)
        T[:3, :3], T[:3, 3] = R, rng.normal(size=3) * 0.3
        poses.append(T)
    poses = np.stack(poses)
    h.tsdf_init(origin, dims, VOX, TRUNC_VOX, 3.0, MAX_W)
    h.tsdf_integrate(dev.data_ptr() + 3 * W * H, 5 * W * H, n, world_T_cam=poses)
    t, w = h.tsdf_read()
    h.close()
    want_t = np.zeros(dims[::-1], dtype=np.float32)
    want_w = np.zeros(dims[::-1], dtype=np.float32)
    for d, T in zip(depth, poses):
        TS.integrate(want_t, want_w, d, _inv(T), (rect.fx, rect.fy, rect.cx, rect.cy), origin, VOX, TRUNC_VOX * VOX,
                     3.0, MAX_W, rect.map_left)
    assert 10000 < (want_w > 0).sum() < 0.5 * want_w.size
    np.testing.assert_array_equal(w, want_w)
    np.testing.assert_array_equal(t, want_t)


@pytest.mark.parametrize("distorted", [False, True])
def test_tsdf_color_layer_bit_exact(distorted):
    """nvblox's colour layer: the record's BGR part integrated with its depth — colour and colour
    weight bit-exact vs the oracle, the TSDF itself unchanged by it."""
    n = 4
    src, rect, h, dev, res, depth = _setup(distorted, n)
    W, H = rect.width, rect.height
    poses = res["T_abs"][:, 0]
    h.tsdf_color(True)
    h.tsdf_init(ORIGIN, DIMS, VOX, TRUNC_VOX, MAX_D, MAX_W)
    h.tsdf_integrate_rgbd(dev.data_ptr(), dev.data_ptr() + 3 * W * H, 5 * W * H, n, world_T_cam=poses)
    t, w = h.tsdf_read()
    col, cw = h.tsdf_read_color()
    rec = dev.cpu().numpy()
    bgr = [rec[f, 0, :3 * W * H].reshape(H, W, 3) for f in range(n)]
    want_t, want_w, want_c, want_cw = _oracle(rect, depth, poses, [True] * n, bgr=bgr)
    np.testing.assert_array_equal(w, want_w)
    np.testing.assert_array_equal(t, want_t)
    assert (want_cw > 0).sum() > 1000 and (want_cw > 0).sum() < (want_w > 0).sum()   # the band only
    np.testing.assert_array_equal(cw, want_cw)
    np.testing.assert_array_equal(col, want_c)
    assert col.max() > 10.0   # real colours, not zeros
    h.close()


def test_engine_dense_map():
    """HipSlamEngine(rgbd, dense_map): each batch's depth integrated with its device-resident tracked
    poses, bit-exact with the oracle on the poses the device tracked; world_T_volume = base_T_rect."""
    from thor_slam_amd.camera import Extrinsics
    from thor_slam_amd.slam.hip_engine import HipSlamEngine

    n = 6
    src = SyntheticRGBDSource(width=320, height=240)
    rig = CameraRig([src], rig_extrinsics={src.name: Extrinsics.from_4x4_matrix(src.rig_T_source)})
    rig.start()
    cfg = HipSlamConfig(rgbd=True, n_features=1000, n_levels=3, batch_size=n, dense_map=True,
                        tsdf_origin=ORIGIN, tsdf_dims=DIMS, tsdf_integrator_max_integration_distance_m=MAX_D,
                        tsdf_max_weight=MAX_W)
    eng = HipSlamEngine(num_cameras=2, config=cfg)
    eng.initialize(rig.calibration)
    depth, bgr = [], []
    for _ in range(n):
        fs = rig.get_synchronized_frames()
        depth.append(np.array(fs.frame_sets[src.name].frames[1].image))
        bgr.append(np.array(fs.frame_sets[src.name].frames[0].image))
        eng.process_frames(fs)
    dm = eng.get_dense_map()
    res = eng.handle.read_poses(n)
    rect = eng.rectifications[0]
    st = res["stats"][:, 0, 0]
    want_t, want_w, want_c, want_cw = _oracle(rect, depth, res["T_abs"][:, 0],
                                              [s == 0 or (s == 2 and f == 0) for f, s in enumerate(st)], bgr=bgr)
    np.testing.assert_array_equal(dm["color_weight"], want_cw)
    np.testing.assert_array_equal(dm["color"], want_c)
    assert (want_w > 0).sum() > 10000
    np.testing.assert_array_equal(dm["weight"], want_w)
    np.testing.assert_array_equal(dm["tsdf"], want_t)
    bt = src.rig_T_source @ src.get_extrinsics()[0].to_4x4_matrix() @ rect.left_optical_T_rect()
    np.testing.assert_allclose(dm["world_T_volume"], bt, atol=1e-12)
    # the dense-map outputs nvblox publishes, from the same volume (oracle/numpy_dense.py)
    from oracle import numpy_dense as DN

    mesh = eng.get_mesh()
    want_m, want_mc = DN.extract_mesh(want_t, want_w, ORIGIN, VOX, cfg.mesh_integrator_min_weight, color=want_c)
    assert want_m.shape[0] > 1000
    np.testing.assert_array_equal(mesh["triangles"].view(np.uint32), want_m.view(np.uint32))
    np.testing.assert_array_equal(mesh["colors"].view(np.uint32), want_mc.view(np.uint32))
    es = eng.get_esdf()
    want_e = DN.esdf(want_t, want_w, VOX, cfg.esdf_integrator_max_distance_m)
    np.testing.assert_array_equal(es["esdf"].view(np.uint32), want_e.view(np.uint32))
    sl = eng.get_esdf_slice()
    y0, y1 = sl["band"]
    assert y1 - y0 == 20
    want_s = DN.esdf_slice(want_t, want_w, VOX, cfg.esdf_integrator_max_distance_m, y0, y1)
    np.testing.assert_array_equal(sl["distance"].view(np.uint32), want_s.view(np.uint32))
    eng.reset()
    assert not eng.get_dense_map()["weight"].any()
    eng.shutdown()


def test_sharded_rgbd_rig_dense_map_equals_one_device():
    """C5 over 4 ranks behind SlamEngine: HipSlamConfig(rgbd, dense_map,
    devices=(0,)*4, copy transport) integrates pair 0's depth and colour on rank 0 with the device
    poses and gives a TSDF, weight and colour layer bit-identical to the one-device engine's."""
    import json
    from pathlib import Path

    from thor_slam_amd.slam.hip_engine import HipSlamEngine
    from thor_slam_amd.synthetic import synthetic_rgbd_rig

    names = ("192.168.2.21", "192.168.2.22", "192.168.2.23", "192.168.2.25")
    joints = json.loads((Path(__file__).parent / "golden" / "brackets_joints.json").read_text())
    n, batch = 8, 4
    sets = None
    out = {}
    for mode, devices in (("one", ()), ("four", (0, 0, 0, 0))):
        srcs, rig = synthetic_rgbd_rig(joints, names, 320, 240)
        rig.start()
        if sets is None:
            sets = [rig.get_synchronized_frames() for _ in range(n)]
        cfg = HipSlamConfig(rgbd=True, n_features=1000, n_levels=3, batch_size=batch, dense_map=True,
                            tsdf_origin=(-7.2, -1.8, -4.4), tsdf_dims=(88, 36, 88), voxel_size=0.1,
                            devices=devices, shard_transport="copy", enable_loop_closure=False)
        eng = HipSlamEngine(num_cameras=8, config=cfg)
        eng.initialize(rig.calibration)
        for fs in sets:
            eng.process_frames(fs)
        dm = eng.get_dense_map()
        out[mode] = (dm, eng._latest_pose.to_4x4_matrix())
        eng.shutdown()
    one, four = out["one"][0], out["four"][0]
    assert (one["weight"] > 0).sum() > 5000
    for key in ("tsdf", "weight", "color", "color_weight"):
        np.testing.assert_array_equal(four[key].view(np.uint32), one[key].view(np.uint32), err_msg=key)
    np.testing.assert_array_equal(out["four"][1], out["one"][1])
