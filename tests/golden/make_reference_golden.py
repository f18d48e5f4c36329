"""Capture golden vectors from the REFERENCE's own code (run only where /root/reference exists).

Imports thor_slam/camera/types.py, rig.py and slam/interface.py directly from the read-only
reference tree (the package __init__ files are bypassed so isaac_ros.py — which needs rclpy/cv2
— is not imported; ``typing.Self`` is aliased because the reference targets Python >= 3.11).
Nothing else is stubbed.  Output: tests/golden/reference_boundary.json.

    python tests/golden/make_reference_golden.py
"""

from __future__ import annotations

import importlib.util
import json
import sys
import types
import typing
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parents[1]
REF = Path("/root/reference")
sys.path[:0] = [str(ROOT), str(ROOT / "thor-slam_amd"), str(ROOT / "tests")]


def load_reference():
    import typing_extensions

    typing.Self = typing_extensions.Self
    for pkg, sub in (("thor_slam", "thor_slam"), ("thor_slam.camera", "thor_slam/camera"), ("thor_slam.slam", "thor_slam/slam")):
        m = types.ModuleType(pkg)
        m.__path__ = [str(REF / sub)]
        sys.modules[pkg] = m
    mods = {}
    for name, rel in (("thor_slam.camera.types", "thor_slam/camera/types.py"), ("thor_slam.camera.rig", "thor_slam/camera/rig.py"),
                      ("thor_slam.slam.interface", "thor_slam/slam/interface.py")):
        spec = importlib.util.spec_from_file_location(name, REF / rel)
        mod = importlib.util.module_from_spec(spec)
        sys.modules[name] = mod
        spec.loader.exec_module(mod)
        mods[name.rsplit(".", 1)[1]] = mod
    return mods


def sync_trace(rig_cls, n_calls: int = 14):
    from helpers import scripted_sources

    rig = rig_cls(scripted_sources(), queue_size=5, imu_source="192.168.2.25")
    rig.start()
    out = []
    for _ in range(n_calls):
        s = rig.get_synchronized_frames()
        if s is None:
            out.append(None)
            continue
        out.append({
            "timestamp": s.timestamp, "max_time_delta": s.max_time_delta,
            "sources": {k: fs.timestamp for k, fs in s.frame_sets.items()},
            "sensor_timestamp": s.sensor_timestamp,
            "accel": None if s.sensor_data is None else list(map(float, s.sensor_data["accelerometer"])),
            "depths": rig.get_queue_depths(),
        })
    latest = rig.get_latest_frames()
    out.append({"latest_timestamp": latest.timestamp, "latest_spread": latest.max_time_delta})
    return out


def world_extrinsics(mods):
    from thor_slam_amd.camera.urdf import CAMERA_MAP, load_rig_extrinsics_from_urdf

    rig_ext = load_rig_extrinsics_from_urdf(REF / "examples/assets/brackets.urdf", CAMERA_MAP)
    T = mods["types"]
    cal = mods["rig"].RigCalibration(
        intrinsics={k: [] for k in CAMERA_MAP},
        extrinsics={k: [T.Extrinsics(np.eye(3), np.array([-0.0375, 0, 0])), T.Extrinsics(np.eye(3), np.array([0.0375, 0, 0]))]
                    for k in CAMERA_MAP},
        rig_extrinsics={k: T.Extrinsics(v.rotation, v.translation) for k, v in rig_ext.items() if k != "192.168.2.23"},
    )
    return {k: [e.to_4x4_matrix().tolist() for e in cal.get_world_extrinsics(k)] for k in sorted(CAMERA_MAP)}


def slampose(mods):
    from scipy.spatial.transform import Rotation

    rng = np.random.default_rng(7)
    sp = mods["interface"].SlamPose
    out = []
    for i in range(6):
        m = np.eye(4)
        m[:3, :3] = Rotation.from_rotvec(rng.normal(0, 1.0, 3)).as_matrix()
        m[:3, 3] = rng.normal(0, 2.0, 3)
        p = sp.from_4x4_matrix(m, timestamp=float(i))
        out.append({"matrix": m.tolist(), "rotation": p.rotation.tolist(), "position": p.position.tolist(),
                    "back": p.to_4x4_matrix().tolist()})
    ident = sp.identity(3.5)
    return {"poses": out, "identity": {"position": ident.position.tolist(), "rotation": ident.rotation.tolist(),
                                       "timestamp": ident.timestamp, "state": ident.tracking_state.name,
                                       "confidence": ident.confidence},
            "states": [s.name for s in mods["interface"].TrackingState],
            "slam_config": {k: getattr(mods["interface"].SlamConfig(), k) for k in mods["interface"].SlamConfig.__dataclass_fields__}}


def main():
    mods = load_reference()
    data = {
        "rig_sync": sync_trace(mods["rig"].CameraRig),
        "world_extrinsics": world_extrinsics(mods),
        "slampose": slampose(mods),
        "source": "reference thor_slam/camera/rig.py, types.py, slam/interface.py @ 2026-01-30",
    }
    (HERE / "reference_boundary.json").write_text(json.dumps(data, indent=1))
    print("wrote", HERE / "reference_boundary.json")


if __name__ == "__main__":
    main()
