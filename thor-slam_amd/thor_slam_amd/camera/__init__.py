"""Camera data model, rig synchronisation and URDF rig loading (reference ``thor_slam.camera``)."""

from .rig import CameraRig, RigCalibration
from .types import (
    CameraFrame,
    CameraSensorType,
    CameraSource,
    Extrinsics,
    FrameSet,
    IMUData,
    IMUExtrinsics,
    Intrinsics,
    IPv4,
    SensorData,
    SynchronizedFrameSet,
)
from .urdf import CAMERA_MAP, load_rig_extrinsics_from_urdf, parse_urdf_transform

__all__ = [
    "CAMERA_MAP",
    "CameraFrame",
    "CameraRig",
    "CameraSensorType",
    "CameraSource",
    "Extrinsics",
    "FrameSet",
    "IMUData",
    "IMUExtrinsics",
    "IPv4",
    "Intrinsics",
    "RigCalibration",
    "SensorData",
    "SynchronizedFrameSet",
    "load_rig_extrinsics_from_urdf",
    "parse_urdf_transform",
]
