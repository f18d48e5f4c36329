"""Sensor data model consumed by the SLAM back end.

API-compatible restatement of ``thor_slam/camera/types.py`` (reference snapshot
2026-01-30).  Field names, field order and semantics are kept identical so that a
``SynchronizedFrameSet`` produced by the reference ``CameraRig`` can be handed to
this package's engines unchanged (and vice versa).  Anchors:

* ``IPv4``                 types.py:13-28
* ``Intrinsics``           types.py:31-38   (K 3x3, distortion coeffs, image size)
* ``Extrinsics``           types.py:41-69   (R 3x3, t in metres; 4x4 helpers)
* ``IMUExtrinsics``        types.py:72-81
* ``CameraFrame``          types.py:84-91   (image is u8 HxW MONO or HxWx3 BGR)
* ``CameraSource`` ABC     types.py:131-210
* ``FrameSet``             types.py:213-254 (timestamp = first frame's, :231-237)
* ``SynchronizedFrameSet`` types.py:257-307
"""

from __future__ import annotations

import re
from abc import ABC, abstractmethod
from dataclasses import dataclass
from typing import Literal

import numpy as np

CameraSensorType = Literal["COLOR", "MONO"]

_IPV4_OCTET = r"(25[0-5]|2[0-4][0-9]|[01]?[0-9][0-9]?)"
_IPV4_RE = re.compile(rf"^({_IPV4_OCTET}\.){{3}}{_IPV4_OCTET}$")


class IPv4(str):
    """A validated dotted-quad address (used as a camera source name)."""

    _ip: str

    def __init__(self, ip: str) -> None:
        if not _IPV4_RE.match(ip):
            raise ValueError(f"Invalid IPv4 address: {ip}")
        self._ip = ip

    def __str__(self) -> str:
        return self._ip

    @property
    def ip(self) -> str:
        return self._ip


@dataclass
class Intrinsics:
    """Pinhole intrinsics at the published image size."""

    width: int
    height: int
    matrix: np.ndarray  # 3x3 K
    coeffs: np.ndarray  # distortion (Luxonis: 14 rational-polynomial coefficients)


@dataclass
class Extrinsics:
    """Rigid transform (rotation 3x3, translation 3 in metres)."""

    rotation: np.ndarray
    translation: np.ndarray

    @classmethod
    def from_4x4_matrix(cls, matrix: np.ndarray | list[list[float]]) -> "Extrinsics":
        m = np.array(matrix)
        if m.shape != (4, 4):
            raise ValueError(f"Expected 4x4 matrix, got shape {m.shape}")
        return cls(rotation=m[:3, :3], translation=m[:3, 3])

    def to_4x4_matrix(self) -> np.ndarray:
        out = np.eye(4)
        out[:3, :3] = self.rotation
        out[:3, 3] = self.translation
        return out


@dataclass
class IMUExtrinsics:
    """IMU pose (in the rig/world frame) and the source that carries the IMU."""

    source_name: str
    extrinsics: Extrinsics

    def to_4x4_matrix(self) -> np.ndarray:
        return self.extrinsics.to_4x4_matrix()


@dataclass
class CameraFrame:
    """One image from one camera."""

    image: np.ndarray
    timestamp: float
    sequence_num: int
    camera_name: str


class SensorData(ABC):
    """Non-image sensor sample (reference types.py:94-110)."""

    @abstractmethod
    def get_timestamp(self) -> float: ...

    @abstractmethod
    def get_sequence_num(self) -> int: ...

    @abstractmethod
    def get_data(self) -> dict: ...


class IMUData(SensorData):
    """Accelerometer [m/s^2] + gyroscope [rad/s] sample (reference types.py:113-128)."""

    accelerometer: np.ndarray
    gyroscope: np.ndarray
    timestamp: float
    sequence_num: int

    def get_timestamp(self) -> float:
        return self.timestamp

    def get_sequence_num(self) -> int:
        return self.sequence_num

    def get_data(self) -> dict:
        return {"accelerometer": self.accelerometer, "gyroscope": self.gyroscope}


class CameraSource(ABC):
    """A device (or synthetic generator) producing frame lists, stereo = [left, right]."""

    @property
    @abstractmethod
    def name(self) -> str: ...

    @abstractmethod
    def start(self) -> None: ...

    @abstractmethod
    def stop(self) -> None: ...

    @abstractmethod
    def get_latest_frames(self) -> list[CameraFrame]:
        """Blocking fetch of the newest frames."""

    @abstractmethod
    def try_get_latest_frames(self) -> list[CameraFrame] | None:
        """Non-blocking fetch; ``None`` when nothing is ready."""

    @abstractmethod
    def get_intrinsics(self) -> list[Intrinsics]: ...

    @abstractmethod
    def get_extrinsics(self) -> list[Extrinsics]: ...

    @abstractmethod
    def get_sensor_extrinsics(self) -> Extrinsics | None: ...

    @abstractmethod
    def get_timestamped_sensor_data(self) -> tuple[dict | None, float | None]: ...

    def try_get_timestamped_sensor_data(self) -> tuple[dict | None, float | None]:
        """Non-blocking sensor read; swallows errors like the reference (types.py:190-204)."""
        if not self.has_sensor_data:
            return None, None
        try:
            return self.get_timestamped_sensor_data()
        except Exception:
            return None, None

    @property
    @abstractmethod
    def has_sensor_data(self) -> bool: ...


@dataclass
class FrameSet:
    """Frames of one source captured together; ``timestamp`` is the first frame's."""

    timestamp: float
    frames: list[CameraFrame]
    source_name: str
    sensor_data: dict | None = None
    sensor_timestamp: float | None = None

    @classmethod
    def from_frames(cls, frames: list[CameraFrame], source_name: str) -> "FrameSet":
        if not frames:
            raise ValueError("Cannot create FrameSet from empty frame list")
        return cls(timestamp=frames[0].timestamp, frames=frames, source_name=source_name)

    def get_timestamps(self) -> list[float]:
        return [f.timestamp for f in self.frames]

    def get_max_timestamp(self) -> float:
        return max(self.get_timestamps())

    def get_min_timestamp(self) -> float:
        return min(self.get_timestamps())

    def get_timestamp_spread(self) -> float:
        ts = self.get_timestamps()
        return max(ts) - min(ts)


@dataclass
class SynchronizedFrameSet:
    """One FrameSet per source, matched to the slowest source's timestamp."""

    timestamp: float
    frame_sets: dict[str, FrameSet]
    max_time_delta: float
    sensor_data: dict | None = None
    sensor_timestamp: float | None = None

    def get_all_frames(self) -> list[CameraFrame]:
        return [f for fs in self.frame_sets.values() for f in fs.frames]

    def get_frames_for_source(self, source_name: str) -> list[CameraFrame] | None:
        fs = self.frame_sets.get(source_name)
        return None if fs is None else fs.frames

    def get_all_timestamps(self) -> dict[str, list[float]]:
        return {name: fs.get_timestamps() for name, fs in self.frame_sets.items()}

    def get_timestamp_for_frame(self, source_name: str, frame_index: int) -> float | None:
        fs = self.frame_sets.get(source_name)
        if fs is None or not 0 <= frame_index < len(fs.frames):
            return None
        return fs.frames[frame_index].timestamp
