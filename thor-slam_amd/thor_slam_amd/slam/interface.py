"""The SLAM engine contract — the drop-in boundary of this back end.

API-compatible restatement of ``thor_slam/slam/interface.py``:

* ``TrackingState``  interface.py:16-23
* ``CameraConfig``   interface.py:26-33  (one entry of the flat, globally indexed camera list)
* ``SlamPose``       interface.py:36-100 (position [x,y,z] m; rotation quaternion [qx,qy,qz,qw]
  in scipy ``as_quat`` order; optional 6x6 covariance ordered translation then rotation)
* ``MapPoint`` / ``SlamMap``  interface.py:103-138
* ``SlamConfig``     interface.py:141-165
* ``SlamEngine``     interface.py:168-270 (ABC; ``process_frames`` may return ``None`` when tracking
  failed, :197-199; save/load/relocalize raise ``NotImplementedError`` by default, :228-256;
  context manager calls ``shutdown``, :259-270)
"""

from __future__ import annotations

from abc import ABC, abstractmethod
from dataclasses import dataclass, field
from enum import Enum, auto

import numpy as np
from scipy.spatial.transform import Rotation

from ..camera.rig import RigCalibration
from ..camera.types import Extrinsics, Intrinsics, SynchronizedFrameSet


class TrackingState(Enum):
    NOT_INITIALIZED = auto()
    INITIALIZING = auto()
    TRACKING = auto()
    LOST = auto()
    RELOCALIZING = auto()


@dataclass
class CameraConfig:
    """One camera of the rig, with its global index given by list position."""

    intrinsics: Intrinsics
    extrinsics: Extrinsics
    source_name: str
    cam_idx: int  # 0 = left, 1 = right for a stereo source


@dataclass
class SlamPose:
    """world_T_body estimate; ``timestamp`` names the frame the pose belongs to."""

    position: np.ndarray
    rotation: np.ndarray
    timestamp: float
    tracking_state: TrackingState = TrackingState.TRACKING
    confidence: float = 1.0
    covariance: np.ndarray | None = None

    def to_4x4_matrix(self) -> np.ndarray:
        m = np.eye(4)
        m[:3, :3] = Rotation.from_quat(self.rotation).as_matrix()
        m[:3, 3] = self.position
        return m

    @classmethod
    def from_4x4_matrix(
        cls,
        matrix: np.ndarray,
        timestamp: float,
        tracking_state: TrackingState = TrackingState.TRACKING,
        confidence: float = 1.0,
    ) -> "SlamPose":
        return cls(
            position=matrix[:3, 3],
            rotation=Rotation.from_matrix(matrix[:3, :3]).as_quat(),
            timestamp=timestamp,
            tracking_state=tracking_state,
            confidence=confidence,
        )

    @classmethod
    def identity(cls, timestamp: float = 0.0) -> "SlamPose":
        return cls(position=np.zeros(3), rotation=np.array([0.0, 0.0, 0.0, 1.0]), timestamp=timestamp)


@dataclass
class MapPoint:
    position: np.ndarray
    color: np.ndarray | None = None
    normal: np.ndarray | None = None
    observations: int = 1


@dataclass
class SlamMap:
    points: list[MapPoint] = field(default_factory=list)
    keyframe_poses: list[SlamPose] = field(default_factory=list)
    timestamp: float = 0.0

    def to_point_cloud(self) -> np.ndarray:
        if not self.points:
            return np.empty((0, 3))
        return np.array([p.position for p in self.points])


@dataclass
class SlamConfig:
    num_cameras: int = 2
    rectified_images: bool = True
    enable_loop_closure: bool = True
    enable_mapping: bool = True
    max_map_size: int = 100000
    expected_fps: float = 30.0


class SlamEngine(ABC):
    """Abstract SLAM back end (context-manager capable)."""

    @abstractmethod
    def initialize(self, calibration: RigCalibration, config: SlamConfig | None = None) -> None:
        """Bind calibration; may allocate GPU resources.  Raises ``RuntimeError`` on failure."""

    @abstractmethod
    def process_frames(self, frame_set: SynchronizedFrameSet) -> SlamPose | None:
        """Consume one synchronised set; return the latest pose or ``None`` if tracking failed."""

    @abstractmethod
    def get_tracking_state(self) -> TrackingState: ...

    @abstractmethod
    def get_map(self) -> SlamMap: ...

    @abstractmethod
    def reset(self) -> None: ...

    @abstractmethod
    def shutdown(self) -> None: ...

    def save_map(self, path: str) -> bool:
        raise NotImplementedError("This SLAM engine does not support map saving")

    def load_map(self, path: str) -> bool:
        raise NotImplementedError("This SLAM engine does not support map loading")

    def relocalize(self) -> bool:
        raise NotImplementedError("This SLAM engine does not support relocalization")

    def __enter__(self) -> "SlamEngine":
        return self

    def __exit__(self, exc_type, exc_val, exc_tb) -> None:  # noqa: ANN001
        self.shutdown()
