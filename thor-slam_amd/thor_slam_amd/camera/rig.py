"""Multi-source synchronisation and rig calibration (the SLAM engine's input producer).

API-compatible restatement of ``thor_slam/camera/rig.py``:

* ``RigCalibration``            rig.py:17-70 (``get_world_extrinsics`` = rig_T_source @ source_T_cam, :35-70)
* ``CameraRig``                 rig.py:73-520
* ``get_synchronized_frames``   rig.py:358-415 — poll every source (serial, blocking), reference
  timestamp = min over sources of the newest queued timestamp (:336-356), per source the queued
  FrameSet closest to it (:299-316, first minimum wins), ``max_time_delta`` = largest |ts - ref|,
  closest IMU sample from the IMU source's queue (:403-407).

The engines in this package only *consume* ``SynchronizedFrameSet``; this class exists so the
harness, the bench and the tests can drive the exact reference synchronisation logic with
synthetic sources, on machines where the reference package itself is absent.
"""

from __future__ import annotations

import logging
from collections import deque
from dataclasses import dataclass, field
from threading import Lock
from typing import Sequence

import numpy as np

from .types import CameraSource, Extrinsics, FrameSet, IMUExtrinsics, Intrinsics, SynchronizedFrameSet

logger = logging.getLogger(__name__)


def _identity_extrinsics() -> Extrinsics:
    return Extrinsics.from_4x4_matrix(np.eye(4))


@dataclass
class RigCalibration:
    """Per-source intrinsics/extrinsics plus each source's pose in the rig frame."""

    intrinsics: dict[str, list[Intrinsics]]
    extrinsics: dict[str, list[Extrinsics]]
    source_names: list[str] = field(default_factory=list)
    rig_extrinsics: dict[str, Extrinsics] = field(default_factory=dict)
    imu_extrinsics: IMUExtrinsics | None = None

    def get_world_extrinsics(self, source_name: str) -> list[Extrinsics] | None:
        """world_T_camera = rig_T_source @ source_T_camera for every camera of a source."""
        cams = self.extrinsics.get(source_name)
        if cams is None:
            return None
        rig = self.rig_extrinsics.get(source_name)
        if rig is None:
            logger.warning("No rig extrinsics defined for source %s, returning camera extrinsics as-is", source_name)
            return cams
        rig_m = rig.to_4x4_matrix()
        return [Extrinsics.from_4x4_matrix(rig_m @ c.to_4x4_matrix()) for c in cams]


class CameraRig:
    """Keeps a bounded queue of FrameSets per source and hands out synchronised sets."""

    def __init__(
        self,
        sources: Sequence[CameraSource],
        queue_size: int = 30,
        rig_extrinsics: dict[str, Extrinsics] | None = None,
        imu_extrinsics: IMUExtrinsics | None = None,
        imu_source: str | None = None,
    ) -> None:
        self.sources: dict[str, CameraSource] = {s.name: s for s in sources}
        self.queue_size = queue_size
        self._frame_queues: dict[str, deque[FrameSet]] = {n: deque(maxlen=queue_size) for n in self.sources}
        self._lock = Lock()
        self._running = False
        self._imu_source = imu_source
        self._imu_queue: deque[tuple[float, dict]] = deque(maxlen=queue_size)

        if imu_source is not None:
            if imu_source not in self.sources:
                raise ValueError(
                    f"IMU source '{imu_source}' not found in sources. Available sources: {list(self.sources)}"
                )
            if not self.sources[imu_source].has_sensor_data:
                raise ValueError(
                    f"IMU source '{imu_source}' does not have sensor data enabled. "
                    "Set read_imu=True when creating the camera source."
                )

        if not rig_extrinsics:
            logger.warning("No rig extrinsics provided, using identity transformation for all sources")
            rig_extrinsics = {n: _identity_extrinsics() for n in self.sources}
        if not imu_extrinsics:
            imu_extrinsics = IMUExtrinsics(source_name=imu_source or "", extrinsics=_identity_extrinsics())
        self._calibration = self._build_calibration(rig_extrinsics, imu_extrinsics)

    # -- lifecycle -----------------------------------------------------------------
    def __enter__(self) -> "CameraRig":
        self.start()
        return self

    def __exit__(self, exc_type, exc_val, exc_tb) -> None:  # noqa: ANN001
        self.stop()

    def start(self) -> None:
        if self._running:
            return
        for s in self.sources.values():
            s.start()
        self._running = True

    def stop(self) -> None:
        if not self._running:
            return
        for s in self.sources.values():
            s.stop()
        self._running = False
        self.clear_queues()

    def is_running(self) -> bool:
        return self._running

    # -- calibration ---------------------------------------------------------------
    def _build_calibration(self, rig_extrinsics: dict[str, Extrinsics], imu_extrinsics: IMUExtrinsics) -> RigCalibration:
        return RigCalibration(
            intrinsics={n: s.get_intrinsics() for n, s in self.sources.items()},
            extrinsics={n: s.get_extrinsics() for n, s in self.sources.items()},
            rig_extrinsics=rig_extrinsics,
            imu_extrinsics=imu_extrinsics,
            source_names=list(self.sources),
        )

    @property
    def calibration(self) -> RigCalibration:
        return self._calibration

    def load_rig_extrinsics(
        self, rig_extrinsics: dict[str, Extrinsics], imu_extrinsics: IMUExtrinsics | None = None
    ) -> None:
        unknown = [n for n in rig_extrinsics if n not in self.sources]
        if unknown:
            raise ValueError(f"Unknown source: {unknown[0]}")
        merged = dict(self._calibration.rig_extrinsics)
        merged.update(rig_extrinsics)
        imu = imu_extrinsics or self._calibration.imu_extrinsics or IMUExtrinsics(
            source_name=self._imu_source or "", extrinsics=_identity_extrinsics()
        )
        self._calibration = self._build_calibration(merged, imu)

    def get_rig_extrinsics(self, source_name: str) -> Extrinsics | None:
        return self._calibration.rig_extrinsics.get(source_name)

    def get_world_extrinsics(self, source_name: str) -> list[Extrinsics] | None:
        return self._calibration.get_world_extrinsics(source_name)

    # -- synchronisation -------------------------------------------------------------
    def _poll_cameras(self) -> None:
        for name, src in self.sources.items():
            if name == self._imu_source:
                data, ts = src.try_get_timestamped_sensor_data()
                if data is not None and ts is not None:
                    self._imu_queue.append((ts, data))
            frames = src.get_latest_frames()
            if frames:
                fs = FrameSet.from_frames(frames, source_name=name)
                with self._lock:
                    self._frame_queues[name].append(fs)

    @staticmethod
    def _find_closest_frame_set(queue: deque[FrameSet], target_timestamp: float) -> FrameSet | None:
        if not queue:
            return None
        return min(queue, key=lambda fs: abs(fs.timestamp - target_timestamp))

    @staticmethod
    def _find_closest_imu_data(
        queue: deque[tuple[float, dict]], target_timestamp: float
    ) -> tuple[float | None, dict | None]:
        if not queue:
            return None, None
        ts, data = min(queue, key=lambda item: abs(item[0] - target_timestamp))
        return ts, data

    def _get_reference_timestamp(self) -> float | None:
        with self._lock:
            newest = []
            for q in self._frame_queues.values():
                if not q:
                    return None
                newest.append(q[-1].timestamp)
        return min(newest)

    def get_synchronized_frames(self, max_wait_ms: float = 100.0) -> SynchronizedFrameSet | None:
        """Poll, pick the slowest source's newest timestamp, match every source to it."""
        if not self._running:
            return None
        self._poll_cameras()
        ref = self._get_reference_timestamp()
        if ref is None:
            logger.warning("No reference timestamp found, not all cameras have frames yet")
            return None
        chosen: dict[str, FrameSet] = {}
        max_dt = 0.0
        with self._lock:
            for name, q in self._frame_queues.items():
                fs = self._find_closest_frame_set(q, ref)
                if fs is None:
                    return None
                chosen[name] = fs
                max_dt = max(max_dt, abs(fs.timestamp - ref))
        sensor_data = sensor_ts = None
        if self._imu_source is not None:
            ts, data = self._find_closest_imu_data(self._imu_queue, ref)
            if data is not None:
                sensor_data, sensor_ts = data, ts
        return SynchronizedFrameSet(
            timestamp=ref, frame_sets=chosen, max_time_delta=max_dt, sensor_data=sensor_data, sensor_timestamp=sensor_ts
        )

    def get_latest_frames(self) -> SynchronizedFrameSet | None:
        """Newest FrameSet of every source, no matching (reference rig.py:417-469)."""
        if not self._running:
            return None
        self._poll_cameras()
        chosen: dict[str, FrameSet] = {}
        with self._lock:
            for name, q in self._frame_queues.items():
                if not q:
                    logger.warning("Camera %s has no frames yet", name)
                    return None
                chosen[name] = q[-1]
        ts = [fs.timestamp for fs in chosen.values()]
        sensor_data = sensor_ts = None
        if self._imu_source is not None and self._imu_queue:
            sensor_ts, sensor_data = self._imu_queue[-1]
        return SynchronizedFrameSet(
            timestamp=max(ts) if ts else 0.0,
            frame_sets=chosen,
            max_time_delta=(max(ts) - min(ts)) if ts else 0.0,
            sensor_data=sensor_data,
            sensor_timestamp=sensor_ts,
        )

    def get_source_names(self) -> list[str]:
        return list(self.sources)

    def get_source(self, name: str) -> CameraSource | None:
        return self.sources.get(name)

    def clear_queues(self) -> None:
        with self._lock:
            for q in self._frame_queues.values():
                q.clear()

    def get_queue_depths(self) -> dict[str, int]:
        with self._lock:
            return {n: len(q) for n, q in self._frame_queues.items()}

    def prune_old_frames(self, max_age_seconds: float = 1.0) -> int:
        with self._lock:
            newest = [q[-1].timestamp for q in self._frame_queues.values() if q]
        if not newest:
            return 0
        cutoff = max(newest) - max_age_seconds
        pruned = 0
        with self._lock:
            for q in self._frame_queues.values():
                while q and q[0].timestamp < cutoff:
                    q.popleft()
                    pruned += 1
        return pruned
