"""Shared fixtures-as-functions for the parity tests (cached per process)."""

from __future__ import annotations

import functools

import numpy as np

from oracle import numpy_slam as O
from thor_slam_amd.calib import extract_cameras, stereo_pairs, stereo_rectify
from thor_slam_amd.camera.rig import CameraRig
from thor_slam_amd.params import HipSlamConfig
from thor_slam_amd.synthetic import SyntheticStereoSource

DISTORTION = np.array([-0.05, 0.01, 0.0005, -0.0003, 0.0, 0.0, 0.0, 0.0])


def make_source(seed: int = 0, width: int = 640, height: int = 400, distorted: bool = False, n_frames: int = 200):
    return SyntheticStereoSource(seed=seed, width=width, height=height, n_frames=n_frames,
                                 distortion=DISTORTION if distorted else None)


def rig_calibration(src):
    return CameraRig([src]).calibration


@functools.lru_cache(maxsize=8)
def scenario(seed: int = 0, n: int = 4, width: int = 640, height: int = 400, distorted: bool = False,
             cfg_items: tuple = ()):
    """Rendered frames + product rectification + oracle run of one stereo sequence."""
    cfg = HipSlamConfig(**dict(cfg_items))
    src = make_source(seed, width, height, distorted)
    cal = rig_calibration(src)
    cams = extract_cameras(cal, 2)
    (li, ri), = stereo_pairs(cams)
    rect = stereo_rectify(cams[li], cams[ri])
    frames = src.render_stereo_sequence(n)
    trk = O.OracleTracker(cfg, dict(fx=rect.fx, fy=rect.fy, cx=rect.cx, cy=rect.cy, baseline=rect.baseline,
                                    map_l=rect.map_left, map_r=rect.map_right))
    results = [trk.step(frames[i, 0], frames[i, 1]) for i in range(n)]
    return {"cfg": cfg, "src": src, "rect": rect, "frames": frames, "oracle": results, "cams": cams}


def rel_frobenius(a: np.ndarray, b: np.ndarray) -> float:
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))
