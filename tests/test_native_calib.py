"""tslam_create_rig's host side (tslam_calib.cpp) against the Python product calibration it
restates (thor_slam_amd/calib.py; isaac_ros.py:138-157, :364-411): pairing, Bouguet rectification
and the 1/32-px remap tables must be byte-identical, through ctypes and through a gcc-built C
caller (tests/c/rig_from_calib.c).  Host code only: no GPU needed."""

import ctypes
import subprocess

import numpy as np
import pytest
from scipy.spatial.transform import Rotation

import native_caller
from helpers import C3_SOURCES, make_source, rig_calibration
from thor_slam_amd._lib import CameraDesc, Params, camera_desc, load_library, make_params, native_rectify_pair
from thor_slam_amd.calib import extract_cameras, rgbd_undistort, stereo_pairs, stereo_rectify
from thor_slam_amd.camera.types import Extrinsics, Intrinsics
from thor_slam_amd.params import HipSlamConfig
from thor_slam_amd.slam.interface import CameraConfig

EINVAL = -1   # TSLAM_EINVAL


def _random_pair(seed: int):
    """A random stereo pair: image size, distortion model (0/2/4/5/7/8/14 coefficients), a rotated
    rig pose, slightly rotated right camera, horizontal or (every 5th) vertical baseline."""
    rng = np.random.default_rng(seed)
    w, h = [(640, 400), (320, 200), (1280, 800), (101, 77)][seed % 4]
    nco = [0, 4, 5, 8, 14, 2, 7][seed % 7]

    def k():
        f = rng.uniform(200, 600)
        return np.array([[f * rng.uniform(0.98, 1.02), 0, w / 2 + rng.uniform(-5, 5)], [0, f, h / 2 + rng.uniform(-5, 5)],
                         [0, 0, 1]])

    base = Rotation.from_euler("xyz", rng.normal(0, 0.5, 3)).as_matrix()
    tb = rng.normal(0, 1, 3)
    rel = Rotation.from_euler("xyz", rng.normal(0, 0.02, 3)).as_matrix()
    bl = np.array([0.075, rng.normal(0, 0.003), rng.normal(0, 0.003)]) if seed % 5 else \
        np.array([rng.normal(0, 0.003), 0.08, 0.0])
    left = CameraConfig(Intrinsics(w, h, k(), rng.normal(0, 0.02, nco)), Extrinsics(base, tb), "s", 0)
    right = CameraConfig(Intrinsics(w, h, k(), rng.normal(0, 0.02, nco)), Extrinsics(base @ rel, tb + base @ bl), "s", 1)
    return left, right


def _assert_same(py, nat, left):
    assert (nat["fx"], nat["fy"], nat["cx"], nat["cy"]) == (py.fx, py.fy, py.cx, py.cy)
    assert abs(nat["baseline"] - py.baseline) <= 1e-14
    np.testing.assert_array_equal(nat["map_left"], py.map_left)
    np.testing.assert_array_equal(nat["map_right"], py.map_right)
    np.testing.assert_allclose(nat["base_T_rect"], left.extrinsics.to_4x4_matrix() @ py.left_optical_T_rect(),
                               rtol=0, atol=1e-13)


@pytest.mark.parametrize("seed", range(12))
def test_rectify_pair_matches_calib(seed):
    left, right = _random_pair(seed)
    py = stereo_rectify(left, right)
    nat = native_rectify_pair(left, right)
    _assert_same(py, nat, left)
    np.testing.assert_allclose(nat["rect_left"], py.rect_left, rtol=0, atol=1e-13)
    np.testing.assert_allclose(nat["rect_right"], py.rect_right, rtol=0, atol=1e-13)


@pytest.mark.parametrize("seed", [0, 3, 4])
def test_rgbd_undistort_matches_calib(seed):
    left, _ = _random_pair(seed)
    py = rgbd_undistort(left)
    nat = native_rectify_pair(left, rgbd=True)
    assert (nat["fx"], nat["fy"], nat["cx"], nat["cy"], nat["baseline"]) == (py.fx, py.fy, py.cx, py.cy, 1.0)
    np.testing.assert_array_equal(nat["map_left"], py.map_left)


def test_identity_rig_gives_identity_tables():
    cams = extract_cameras(rig_calibration(make_source(distorted=False)), 2)
    nat = native_rectify_pair(cams[0], cams[1])
    assert stereo_rectify(cams[0], cams[1]).is_identity
    ident = np.stack(np.meshgrid(np.arange(640), np.arange(400)), axis=-1).astype(np.int32) * 32
    np.testing.assert_array_equal(nat["map_left"], ident)


def test_rig_pairs_follow_extract_cameras_order():
    """Sources are taken in sorted name order whatever order the caller lists them in."""
    lib = load_library()
    k = np.array([[400.0, 0, 320], [0, 400, 200], [0, 0, 1]])
    spec = [("b", 0), ("a", 1), ("b", 1), ("a", 0), ("c", 0)]   # a's cameras listed out of cam_idx order
    cams = [CameraConfig(Intrinsics(640, 400, k, np.zeros(5)), Extrinsics(np.eye(3), np.zeros(3)), s, i) for s, i in spec]
    descs = (CameraDesc * len(cams))(*[camera_desc(c) for c in cams])
    out = (ctypes.c_int32 * 8)()
    assert lib.tslam_rig_pairs(descs, len(cams), out, 4) == 1   # a: [1, 3] is (1, 0) -> no pair; b: (0, 2)
    assert list(out[:2]) == [0, 2]
    ordered = [cams[i] for i in (3, 1, 0, 2, 4)]   # a0 a1 b0 b1 c0: what extract_cameras yields
    d2 = (CameraDesc * 5)(*[camera_desc(c) for c in ordered])
    assert lib.tslam_rig_pairs(d2, 5, out, 4) == 2
    assert [tuple(out[2 * p:2 * p + 2]) for p in range(2)] == [(0, 1), (2, 3)] == stereo_pairs(ordered)


def test_create_rig_argument_errors():
    """EINVAL paths of tslam_create_rig that are decided on the host before any device work."""
    lib = load_library()
    k = np.array([[400.0, 0, 320], [0, 400, 200], [0, 0, 1]])
    mono = [CameraConfig(Intrinsics(640, 400, k, np.zeros(5)), Extrinsics(np.eye(3), np.zeros(3)), "s", 0)]
    descs = (CameraDesc * 1)(*[camera_desc(c) for c in mono])
    params = make_params(HipSlamConfig(), 4, 0, 0)
    h = ctypes.c_void_p()
    assert lib.tslam_create_rig(descs, 1, ctypes.byref(params), 0, ctypes.byref(h)) == EINVAL
    assert b"no stereo source" in lib.tslam_last_error()
    left, right = _random_pair(1)
    d2 = (CameraDesc * 2)(camera_desc(left), camera_desc(right))
    params = make_params(HipSlamConfig(), 4, 3, 0)   # n_pairs disagrees with the one pair found
    assert lib.tslam_create_rig(d2, 2, ctypes.byref(params), 0, ctypes.byref(h)) == EINVAL
    assert isinstance(params, Params)


def test_c_caller_tables_match_calib(tmp_path):
    """The gcc-built C caller produces, for the C3 brackets rig (4 sources, rotated mounts) and a
    distorted pair, the very bytes HipSlamEngine.initialize builds in Python."""
    from helpers import rig_scene

    exe = native_caller.build()
    for cams in (rig_scene(names=C3_SOURCES, n=1)["cams"],
                 extract_cameras(rig_calibration(make_source(distorted=True)), 2)):
        native_caller.write_calib(cams, tmp_path / "calib.txt")
        subprocess.run([str(exe), "maps", str(tmp_path / "calib.txt"), str(tmp_path / "maps.bin")], check=True)
        pairs = stereo_pairs(cams)
        got = native_caller.read_maps(tmp_path / "maps.bin", len(pairs), 640, 400)
        for (l, r), g in zip(pairs, got):
            assert g["pair"] == (l, r)
            _assert_same(stereo_rectify(cams[l], cams[r]), g, cams[l])
