"""RGB-D input records (BASELINE.json configs[4]).

A Luxonis RGB-D source yields (colour BGR u8 H x W x 3, depth u16 mm H x W aligned to the colour
camera) per frame (``get_latest_rgbd_frames``, thor_slam/camera/drivers/luxonis.py:876-919).  The
device reads one contiguous record per camera and frame: the BGR bytes followed by the depth bytes.
"""

from __future__ import annotations

import numpy as np


def pack_rgbd(bgr: np.ndarray, depth: np.ndarray) -> np.ndarray:
    """One RGB-D record as the device reads it: BGR u8 bytes followed by the u16 depth bytes."""
    return np.concatenate([np.ascontiguousarray(bgr, dtype=np.uint8).reshape(-1),
                           np.ascontiguousarray(depth, dtype="<u2").view(np.uint8).reshape(-1)])


def unpack_rgbd(record: np.ndarray, width: int, height: int) -> tuple[np.ndarray, np.ndarray]:
    """Inverse of ``pack_rgbd``: (BGR u8 H x W x 3, depth u16 H x W) views of one record."""
    rec = np.ascontiguousarray(record, dtype=np.uint8).reshape(-1)
    n = width * height
    return rec[:3 * n].reshape(height, width, 3), rec[3 * n:5 * n].view("<u2").reshape(height, width)
