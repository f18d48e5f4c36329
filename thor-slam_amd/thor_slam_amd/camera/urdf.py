"""URDF star-topology rig loader (builds ``rig_extrinsics`` for multi-source rigs, config C3).

Restates the pure-math part of ``thor_slam/camera/utils.py``:

* ``parse_urdf_transform``          utils.py:101-126 — ``xyz`` + ``rpy`` of a fixed joint's
  ``<origin>``.  NOTE: the reference converts rpy with scipy ``from_euler("XYZ", ...)``, i.e.
  *intrinsic* X-Y-Z, although its comment says extrinsic (utils.py:116-118).  We replicate the
  reference behaviour, not the comment, so rig extrinsics match bit for bit.
* ``load_rig_extrinsics_from_urdf`` utils.py:129-178 — for each source, the first joint whose
  child link matches and whose parent is ``base_link``.

The DepthAI device helpers of utils.py are hardware I/O and out of scope.
"""

from __future__ import annotations

import logging
import xml.etree.ElementTree as ET
from pathlib import Path

import numpy as np
from scipy.spatial.transform import Rotation

from .types import Extrinsics

logger = logging.getLogger(__name__)

# Reference CAMERA_MAP (scripts/run_slam.py:45-50): source IP -> URDF link.
CAMERA_MAP = {
    "192.168.2.25": "link_Camera_1_centroid",
    "192.168.2.21": "link_Camera_2_centroid",
    "192.168.2.23": "link_Camera_3_centroid",
    "192.168.2.22": "link_Camera_4_centroid",
}


def parse_urdf_transform(joint_elem: ET.Element) -> np.ndarray:
    """4x4 parent_T_child of a fixed joint (identity when ``<origin>`` is absent)."""
    origin = joint_elem.find("origin")
    if origin is None:
        logger.warning("Joint %s has no origin tag, assuming identity.", joint_elem.get("name"))
        return np.eye(4)
    xyz = np.array([float(v) for v in origin.get("xyz", "0 0 0").split()])
    rpy = [float(v) for v in origin.get("rpy", "0 0 0").split()]
    out = np.eye(4)
    out[:3, :3] = Rotation.from_euler("XYZ", rpy, degrees=False).as_matrix()
    out[:3, 3] = xyz
    return out


def load_rig_extrinsics_from_urdf(urdf_path: str | Path, camera_map: dict[str, str]) -> dict[str, Extrinsics]:
    """Source name -> base_link_T_source for every mapped link directly under base_link."""
    urdf_path = Path(urdf_path)
    if not urdf_path.exists():
        raise FileNotFoundError(f"URDF not found at {urdf_path}")
    joints = ET.parse(urdf_path).getroot().findall("joint")
    out: dict[str, Extrinsics] = {}
    for source, link in camera_map.items():
        for joint in joints:
            child = joint.find("child")
            if child is None or child.get("link") != link:
                continue
            parent = joint.find("parent")
            if parent is None or parent.get("link") != "base_link":
                logger.warning("Skipping joint %s: parent is not base_link", joint.get("name"))
                continue
            out[source] = Extrinsics.from_4x4_matrix(parse_urdf_transform(joint))
            break
        else:
            logger.warning("Could not find URDF link matching '%s' for source %s", link, source)
    return out
