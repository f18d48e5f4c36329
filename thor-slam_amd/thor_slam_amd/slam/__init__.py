"""SLAM boundary (reference ``thor_slam.slam``) and the MI355X engine."""

from .interface import CameraConfig, MapPoint, SlamConfig, SlamEngine, SlamMap, SlamPose, TrackingState

__all__ = ["CameraConfig", "MapPoint", "SlamConfig", "SlamEngine", "SlamMap", "SlamPose", "TrackingState"]
