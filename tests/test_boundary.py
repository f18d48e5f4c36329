"""The restated boundary (types, CameraRig, RigCalibration, SlamPose, SlamEngine contract) against
golden vectors captured from the reference's own code (tests/golden/make_reference_golden.py),
plus live comparisons when /root/reference is present (build container only)."""

import json
import math
from pathlib import Path

import numpy as np
import pytest
from scipy.spatial.transform import Rotation

from helpers import scripted_sources
from thor_slam_amd.camera import CAMERA_MAP, CameraRig, Extrinsics, FrameSet, RigCalibration, load_rig_extrinsics_from_urdf
from thor_slam_amd.camera.urdf import parse_urdf_transform
from thor_slam_amd.slam import SlamConfig, SlamEngine, SlamMap, SlamPose, TrackingState

GOLD = json.loads((Path(__file__).parent / "golden" / "reference_boundary.json").read_text())
REF = Path("/root/reference")
URDF = Path(__file__).parent / "golden" / "brackets_joints.json"


def _trace(rig_cls):
    import sys

    sys.path.insert(0, str(Path(__file__).parent / "golden"))
    from make_reference_golden import sync_trace

    return sync_trace(rig_cls)


def test_rig_sync_matches_reference_trace():
    got = _trace(CameraRig)
    assert got == GOLD["rig_sync"]


def test_world_extrinsics_match_reference():
    rig_ext = {k: Extrinsics.from_4x4_matrix(np.array(v)) for k, v in json.loads(URDF.read_text()).items()}
    cal = RigCalibration(
        intrinsics={k: [] for k in CAMERA_MAP},
        extrinsics={k: [Extrinsics(np.eye(3), np.array([-0.0375, 0, 0])), Extrinsics(np.eye(3), np.array([0.0375, 0, 0]))] for k in CAMERA_MAP},
        rig_extrinsics={k: v for k, v in rig_ext.items() if k != "192.168.2.23"},
    )
    for k, mats in GOLD["world_extrinsics"].items():
        got = [e.to_4x4_matrix() for e in cal.get_world_extrinsics(k)]
        np.testing.assert_array_equal(np.array(got), np.array(mats))
    assert cal.get_world_extrinsics("nope") is None


def test_slampose_conventions_match_reference():
    sp = GOLD["slampose"]
    for rec in sp["poses"]:
        p = SlamPose.from_4x4_matrix(np.array(rec["matrix"]), timestamp=0.0)
        np.testing.assert_array_equal(p.rotation, rec["rotation"])
        np.testing.assert_array_equal(p.position, rec["position"])
        np.testing.assert_array_equal(p.to_4x4_matrix(), rec["back"])
    ident = SlamPose.identity(3.5)
    assert ident.rotation.tolist() == sp["identity"]["rotation"] and ident.timestamp == 3.5
    assert ident.tracking_state.name == sp["identity"]["state"] and ident.confidence == 1.0
    assert [s.name for s in TrackingState] == sp["states"]
    cfg = SlamConfig()
    for k, v in sp["slam_config"].items():
        assert getattr(cfg, k) == v


def test_urdf_loader_uses_intrinsic_xyz():
    """Hand-derived pin of utils.py:101-126: rpy -> Rx(r) @ Ry(p) @ Rz(y) (scipy 'XYZ' = intrinsic)."""
    import xml.etree.ElementTree as ET

    j = ET.fromstring('<joint name="j"><origin xyz="0.1 -0.2 0.3" rpy="0.3 -0.7 1.1"/></joint>')
    m = parse_urdf_transform(j)
    r, p, y = 0.3, -0.7, 1.1
    rx = np.array([[1, 0, 0], [0, math.cos(r), -math.sin(r)], [0, math.sin(r), math.cos(r)]])
    ry = np.array([[math.cos(p), 0, math.sin(p)], [0, 1, 0], [-math.sin(p), 0, math.cos(p)]])
    rz = np.array([[math.cos(y), -math.sin(y), 0], [math.sin(y), math.cos(y), 0], [0, 0, 1]])
    np.testing.assert_allclose(m[:3, :3], rx @ ry @ rz, atol=1e-12)
    np.testing.assert_allclose(m[:3, 3], [0.1, -0.2, 0.3])
    assert np.array_equal(parse_urdf_transform(ET.fromstring('<joint name="k"/>')), np.eye(4))


def test_urdf_fixture_loads_four_cameras():
    urdf = REF / "examples/assets/brackets.urdf"
    if not urdf.exists():
        pytest.skip("reference URDF not present (GPU box)")
    ext = load_rig_extrinsics_from_urdf(urdf, CAMERA_MAP)
    assert sorted(ext) == sorted(CAMERA_MAP)
    fixture = json.loads(URDF.read_text())
    for k, e in ext.items():
        np.testing.assert_array_equal(e.to_4x4_matrix(), np.array(fixture[k]))
    # Camera_1 centroid from brackets.urdf:122-125
    np.testing.assert_allclose(ext["192.168.2.25"].translation, [0.00021709, -0.04467888, 0.05586718])
    with pytest.raises(FileNotFoundError):
        load_rig_extrinsics_from_urdf("/nonexistent.urdf", CAMERA_MAP)


def test_frameset_helpers():
    from thor_slam_amd.camera import CameraFrame, SynchronizedFrameSet

    f = [CameraFrame(np.zeros((2, 2), np.uint8), 1.0, 0, "a"), CameraFrame(np.zeros((2, 2), np.uint8), 1.5, 0, "b")]
    fs = FrameSet.from_frames(f, "s")
    assert fs.timestamp == 1.0 and fs.get_timestamp_spread() == 0.5 and fs.get_max_timestamp() == 1.5
    with pytest.raises(ValueError):
        FrameSet.from_frames([], "s")
    sfs = SynchronizedFrameSet(1.0, {"s": fs}, 0.0)
    assert sfs.get_timestamp_for_frame("s", 1) == 1.5 and sfs.get_timestamp_for_frame("s", 2) is None
    assert sfs.get_frames_for_source("x") is None and len(sfs.get_all_frames()) == 2
    assert SlamMap().to_point_cloud().shape == (0, 3)


def test_engine_contract_defaults():
    from thor_slam_amd.slam.hip_engine import HipSlamEngine

    eng = HipSlamEngine(num_cameras=2)
    assert eng.get_tracking_state() == TrackingState.NOT_INITIALIZED
    with pytest.raises(RuntimeError, match="Not initialized"):
        eng.process_frames(None)
    assert eng.save_map("x") is False           # implemented (§8f item 3): nothing mapped yet
    with pytest.raises(RuntimeError, match="Not initialized"):
        eng.relocalize()
    with eng as e:
        assert isinstance(e, SlamEngine)
    assert eng.get_tracking_state() == TrackingState.NOT_INITIALIZED


def test_rig_rejects_bad_imu_source():
    with pytest.raises(ValueError):
        CameraRig(scripted_sources(), imu_source="10.0.0.1")
    with pytest.raises(ValueError):
        CameraRig(scripted_sources(), imu_source="192.168.2.21")


# ------------------------------------------------------------------------------------------------
# live comparisons against the reference code (build container only)
# ------------------------------------------------------------------------------------------------
@pytest.fixture(scope="module")
def ref_mods():
    if not (REF / "thor_slam").exists():
        pytest.skip("/root/reference not present")
    import sys

    sys.path.insert(0, str(Path(__file__).parent / "golden"))
    from make_reference_golden import load_reference

    return load_reference()


def test_live_reference_rig_sync(ref_mods):
    assert _trace(ref_mods["rig"].CameraRig) == _trace(CameraRig)


def test_live_reference_slampose_random(ref_mods):
    rng = np.random.default_rng(11)
    for _ in range(20):
        m = np.eye(4)
        m[:3, :3] = Rotation.from_rotvec(rng.normal(0, 2.0, 3)).as_matrix()
        m[:3, 3] = rng.normal(size=3)
        a = ref_mods["interface"].SlamPose.from_4x4_matrix(m, 1.0)
        b = SlamPose.from_4x4_matrix(m, 1.0)
        np.testing.assert_array_equal(a.rotation, b.rotation)
        np.testing.assert_array_equal(a.to_4x4_matrix(), b.to_4x4_matrix())


def test_fast_quaternion_equals_scipy():
    """The publish path's quaternion (hip_engine._quat_xyzw) is scipy's from_matrix(...).as_quat(),
    bit for bit, on rotations of every branch (trace and each diagonal element the largest)."""
    from scipy.spatial.transform import Rotation

    from thor_slam_amd.slam.hip_engine import _quat_xyzw

    rng = np.random.default_rng(0)
    mats = [Rotation.from_rotvec(rng.normal(0, 1.5, 3)).as_matrix() for _ in range(3000)]
    mats += [Rotation.from_rotvec(np.pi * np.eye(3)[a] * 0.999).as_matrix() for a in range(3)] + [np.eye(3)]
    for m in mats:
        np.testing.assert_array_equal(_quat_xyzw(m), Rotation.from_matrix(m).as_quat())
