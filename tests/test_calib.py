"""Calibration semantics at the boundary (isaac_ros.py:138-157, :370-383, :387-408, :312) and the
rectification tables (product host code vs the oracle's independent derivation)."""

import numpy as np
import pytest
from scipy.spatial.transform import Rotation

from helpers import DISTORTION, make_source, rig_calibration
from oracle import numpy_slam as O
from thor_slam_amd.calib import (
    confidence_from_covariance, distortion_model, extract_cameras, stereo_pairs, stereo_projection, stereo_rectify,
)
from thor_slam_amd.camera.rig import RigCalibration
from thor_slam_amd.camera.types import Extrinsics, Intrinsics


def _cal_two_sources():
    k = np.array([[400.0, 0, 320], [0, 400, 200], [0, 0, 1]])
    intr = lambda: Intrinsics(640, 400, k.copy(), np.zeros(14))  # noqa: E731
    ext = [Extrinsics(np.eye(3), np.array([-0.0375, 0, 0])), Extrinsics(np.eye(3), np.array([0.0375, 0, 0]))]
    return RigCalibration(
        intrinsics={"192.168.2.25": [intr(), intr()], "192.168.2.21": [intr(), intr()]},
        extrinsics={"192.168.2.25": ext, "192.168.2.21": ext},
        rig_extrinsics={"192.168.2.21": Extrinsics(np.eye(3), np.array([1.0, 0, 0]))},
    )


def test_camera_order_sorted_sources_then_cam_idx():
    cams = extract_cameras(_cal_two_sources(), 4)
    assert [(c.source_name, c.cam_idx) for c in cams] == [
        ("192.168.2.21", 0), ("192.168.2.21", 1), ("192.168.2.25", 0), ("192.168.2.25", 1)]
    # world extrinsics applied for a source with rig extrinsics, raw for the other
    np.testing.assert_allclose(cams[0].extrinsics.translation, [0.9625, 0, 0])
    np.testing.assert_allclose(cams[2].extrinsics.translation, [-0.0375, 0, 0])
    assert stereo_pairs(cams) == [(0, 1), (2, 3)]
    assert len(extract_cameras(_cal_two_sources(), 3)) == 3


def test_distortion_model_selection():
    assert distortion_model(np.arange(14.0)) == ("rational_polynomial", list(np.arange(8.0)))
    assert distortion_model(np.arange(5.0))[0] == "plumb_bob"
    assert distortion_model(np.arange(4.0))[0] == "equidistant"
    assert distortion_model(np.arange(2.0)) == ("plumb_bob", [0.0, 1.0, 0.0, 0.0, 0.0])


def test_stereo_projection_baseline():
    cams = extract_cameras(_cal_two_sources(), 2)
    p, b = stereo_projection(cams[0], cams[1])
    assert b == pytest.approx(0.075)
    assert p[0, 3] == pytest.approx(-400.0 * 0.075)


def test_confidence():
    assert confidence_from_covariance(np.zeros((6, 6))) == 1.0
    assert confidence_from_covariance(np.eye(6)) == pytest.approx(0.25)
    assert confidence_from_covariance(None) == 1.0


@pytest.mark.parametrize("distorted", [False, True])
def test_rectification_maps_match_oracle(distorted):
    src = make_source(distorted=distorted)
    cams = extract_cameras(rig_calibration(src), 2)
    r = stereo_rectify(cams[0], cams[1])
    wl, wr = cams[0].extrinsics.to_4x4_matrix(), cams[1].extrinsics.to_4x4_matrix()
    fx, fy, cx, cy, b, ml, mr = O.rectification(cams[0].intrinsics.matrix, cams[0].intrinsics.coeffs, wl,
                                                cams[1].intrinsics.matrix, cams[1].intrinsics.coeffs, wr, 640, 400)
    assert (r.fx, r.fy, r.cx, r.cy) == (fx, fy, cx, cy)
    assert r.baseline == pytest.approx(b) and r.baseline == pytest.approx(0.075)
    np.testing.assert_array_equal(r.map_left, ml)
    np.testing.assert_array_equal(r.map_right, mr)
    assert r.is_identity == (not distorted)


def test_rectification_of_a_rotated_pair_aligns_epipolar_lines():
    k = np.array([[380.0, 0, 319.5], [0, 381, 199.5], [0, 0, 1]])
    rot = Rotation.from_euler("xyz", [0.01, -0.02, 0.015]).as_matrix()
    left = Extrinsics(np.eye(3), np.zeros(3))
    right = Extrinsics(rot, np.array([0.075, 0.002, -0.001]))
    cal = RigCalibration(intrinsics={"s": [Intrinsics(640, 400, k, np.zeros(14)), Intrinsics(640, 400, k, np.zeros(14))]},
                         extrinsics={"s": [left, right]})
    cams = extract_cameras(cal, 2)
    r = stereo_rectify(cams[0], cams[1])
    # a 3D point projects to the same rectified row in both cameras
    pts = np.array([[0.3, -0.2, 2.0], [-1.0, 0.5, 5.0], [0.0, 0.0, 1.0]])
    l_T_r = np.linalg.inv(left.to_4x4_matrix()) @ right.to_4x4_matrix()
    for p in pts:
        pl = r.rect_left @ p
        pr = r.rect_right @ (l_T_r[:3, :3].T @ (p - l_T_r[:3, 3]))
        yl = r.fy * pl[1] / pl[2] + r.cy
        yr = r.fy * pr[1] / pr[2] + r.cy
        assert abs(yl - yr) < 1e-9
        assert r.fx * pl[0] / pl[2] - r.fx * pr[0] / pr[2] > 0  # positive disparity


def test_distorted_render_is_undistorted_by_rectify():
    """Remapping a distorted render approximately reproduces the undistorted render."""
    a = make_source(distorted=False)
    b = make_source(distorted=True)
    cams = extract_cameras(rig_calibration(b), 2)
    r = stereo_rectify(cams[0], cams[1])
    img_u = a.scene.render(a.camera_pose(0, 0), a.get_intrinsics()[0], None)
    img_d = b.scene.render(b.camera_pose(0, 0), b.get_intrinsics()[0], None)
    rect = O.remap(img_d, r.map_left).astype(float)
    inner = (slice(40, 360), slice(60, 580))
    assert np.mean(np.abs(rect[inner] - img_u[inner].astype(float))) < 6.0
    assert np.mean(np.abs(img_d[inner].astype(float) - img_u[inner].astype(float))) > 10.0
    assert DISTORTION[0] != 0
