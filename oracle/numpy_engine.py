"""BASELINE.json configs[0] — the NumPy CPU ``SlamEngine``.

TEST INFRASTRUCTURE (see ``oracle/__init__.py``): the CPU reference engine of SURVEY.md §7 step 2
("``NumpySlamEngine(SlamEngine)``"), timed by ``bench.py``'s ``cpu_baseline`` leg and run by
``tests/test_numpy_engine.py``.  The product never imports it.

It drops in behind ``thor_slam.slam.interface.SlamEngine`` exactly like ``HipSlamEngine`` (the
reference's loop ``scripts/run_slam.py:299-328``: ``initialize(rig.calibration)``, then
``process_frames`` per ``SynchronizedFrameSet``) and runs the oracle of every row, one frame at a
time (the batch-1 semantics of the GPU engine's default path):

* camera order / stereo pairs / rectification: the boundary layer (``thor_slam_amd.calib``, pinned
  against the reference's own ``isaac_ros.py`` rules), as every parity test feeds the oracle;
* A2-A7 per pair: ``numpy_slam.OracleTracker``; several pairs: ``numpy_rig.rig_pose`` and the body
  chain (``numpy_imu.run_rig_sequence``'s rule);
* A8 local BA (``ba_window`` > 0, one pair): ``numpy_ba.BATracker``, the published pose the front
  end carried by the newest keyframe's correction (``HipSlamEngine._ba_corrections``);
* IMU fusion when the calibration carries the IMU: ``numpy_imu.ImuFilter`` with the lagged priors
  of ``imu_prior_lag`` (``lagged_priors``), one pair;
* loop closure (``enable_loop_closure``, one pair): ``numpy_loop.LoopPolicy`` over a keyframe
  database of ``keyframe_landmarks`` with ``vote`` / ``verify`` / ``optimize``.
"""

from __future__ import annotations

import numpy as np

from . import numpy_slam as O
from .numpy_ba import BAParams, BATracker
from .numpy_imu import ImuFilter, lagged_priors, vision_only
from .numpy_loop import LoopPolicy, keyframe_landmarks, optimize, verify, vote
from .numpy_rig import inv_rigid, rig_pose

from thor_slam_amd.slam.interface import SlamEngine   # the boundary's ABC (restates interface.py:168-270)


def _quat(R: np.ndarray) -> np.ndarray:
    from scipy.spatial.transform import Rotation

    return Rotation.from_matrix(R).as_quat()


class NumpySlamEngine(SlamEngine):
    """The CPU reference ``SlamEngine``."""

    def __init__(self, num_cameras: int = 2, config=None) -> None:
        from thor_slam_amd.params import HipSlamConfig
        from thor_slam_amd.slam.interface import TrackingState

        self._num_cameras = num_cameras
        self._config = config or HipSlamConfig(num_cameras=num_cameras)
        self._TS = TrackingState
        self._state = TrackingState.NOT_INITIALIZED
        self._trackers: list = []
        self._latest = None
        self.frame_count = 0
        self.results: list = []   # per frame: the trackers' results (tests)

    # -- SlamEngine ------------------------------------------------------------------------------
    def initialize(self, calibration, config=None) -> None:
        from thor_slam_amd.calib import extract_cameras, stereo_pairs, stereo_rectify
        from thor_slam_amd.params import HipSlamConfig

        if isinstance(config, HipSlamConfig):
            self._config = config
        cfg = self._config
        self._cameras = extract_cameras(calibration, self._num_cameras)
        self._pairs = stereo_pairs(self._cameras)
        if not self._pairs:
            raise RuntimeError("NumpySlamEngine needs at least one stereo source (cam_idx 0 and 1)")
        self._rects = [stereo_rectify(self._cameras[l], self._cameras[r]) for l, r in self._pairs]
        self._E = [self._cameras[l].extrinsics.to_4x4_matrix() @ r.left_optical_T_rect()
                   for (l, _), r in zip(self._pairs, self._rects)]
        self._rect_d = [dict(fx=r.fx, fy=r.fy, cx=r.cx, cy=r.cy, baseline=r.baseline, map_l=r.map_left,
                             map_r=r.map_right) for r in self._rects]
        imu = getattr(calibration, "imu_extrinsics", None)
        self._base_T_imu = imu.to_4x4_matrix() if imu is not None else None
        self._fusion = cfg.imu_fusion if cfg.imu_fusion is not None else imu is not None
        self._reset_state()
        self._state = self._TS.INITIALIZING

    def _reset_state(self) -> None:
        cfg, P = self._config, len(self._pairs)
        self._trackers = [O.OracleTracker(cfg, d) for d in self._rect_d]
        self._T_body = np.eye(4)   # the rig's chained body pose (world = base_link at frame 0)
        self._g = 0
        self._latest = None
        self._ba = None
        if cfg.ba_window > 0 and P == 1:
            d = self._rect_d[0]
            self._ba = BATracker(cfg.n_features, (d["fx"], d["fy"], d["cx"], d["cy"], d["fx"] * d["baseline"]),
                                 BAParams(cfg.ba_window, cfg.ba_kf_interval, cfg.ba_iters, cfg.ba_lambda,
                                          cfg.ba_outlier_px))
        self._fe_at = {}
        self._filt = None
        if self._fusion and P == 1:
            rect_T_imu = inv_rigid(self._E[0]) @ (self._base_T_imu if self._base_T_imu is not None else np.eye(4))
            self._filt = ImuFilter(rect_T_imu[:3, :3], cfg.accelerometer_noise_density, cfg.accelerometer_random_walk,
                                   cfg.gyroscope_noise_density, cfg.gyroscope_random_walk, cfg.imu_rot_floor,
                                   cfg.imu_trans_floor, ba0_sigma=cfg.imu_accel_bias_sigma,
                                   bg0_sigma=cfg.imu_gyro_bias_sigma, lever=rect_T_imu[:3, 3],
                                   accel=cfg.imu_accel if cfg.imu_accel is not None else True,
                                   vis_rot_floor=cfg.imu_vis_rot_floor)
        self._pending = []       # tracked frames whose vision the filter has not absorbed: (n, [(i, res, prior)], [sample])
        self._prev_ts = None
        self._loop = None
        if cfg.enable_loop_closure and P == 1:
            d = self._rect_d[0]
            self._intr = (d["fx"], d["fy"], d["cx"], d["cy"], d["fx"] * d["baseline"])
            self._db: dict[int, dict] = {}   # database position -> landmarks (+ the frame's features)
            self._loop = LoopPolicy(cfg, 1, [np.eye(4)], self._vote, self._verify,
                                    lambda T, e, m, i, it: optimize(T, e, m, i, it))
        self.results = []

    # database of the loop policy (positions = node indices, a ring of loop_max_keyframes)
    def _vote(self, idx, q, lo, n):
        cfg = self._config
        qd = self._db[idx % cfg.loop_max_keyframes]["desc"]
        return np.array([vote(qd, self._db[c % cfg.loop_max_keyframes]["desc"], cfg.loop_signature, cfg.max_hamming,
                              cfg.ratio_pct) for c in range(lo, lo + n)])

    def _verify(self, idx, g, q, c, pc):
        cfg = self._config
        o = verify(self._db[idx % cfg.loop_max_keyframes]["feat"], self._db[c % cfg.loop_max_keyframes],
                   self._intr[:4], cfg, g)
        st = np.zeros(8, dtype=np.int32)
        st[0], st[1], st[2] = int(o["status"]), int(o.get("n_corr", 0)), int(o.get("n_inliers", 0))
        return {"T": o["T"], "stats": st}

    def _imu_priors(self, ts: float, sample) -> tuple | None:
        """The frame's IMU prior with imu_prior_lag frames' vision not yet absorbed (batch 1)."""
        filt, lag = self._filt, max(int(self._config.imu_prior_lag), 0)
        while self._pending and self._pending[0][0] <= self._g - 1 - lag:
            for i, r, pr in self._pending.pop(0)[1]:
                dt, gy, ac = self._samples[i]
                if dt is None:
                    continue
                T, C = r["T"], r["cov"]
                if int(r["status"]) == 0 and pr is not None:
                    T, C = vision_only(T, C, r["sigma2"], pr)
                filt.update(filt.predict(dt, gy, ac), int(r["status"]), T, C)
        if sample is None:
            smp = (None, None, None)
        else:
            if not filt.ready:
                filt.start(sample[1])
                smp = (None, sample[0], sample[1])
            else:
                smp = (ts - self._prev_ts if self._prev_ts is not None and ts > self._prev_ts else None,
                       sample[0], sample[1])
        self._samples[self._g] = smp
        return smp

    def process_frames(self, frame_set):
        if not self._trackers:
            raise RuntimeError("Not initialized")
        self.frame_count += 1
        imgs = []
        for l, r in self._pairs:
            for gi in (l, r):
                cam = self._cameras[gi]
                fs = frame_set.frame_sets.get(cam.source_name)
                if fs is None or cam.cam_idx >= len(fs.frames):
                    return self._latest
                img = np.asarray(fs.frames[cam.cam_idx].image)
                imgs.append(img if img.ndim == 2 else O.bgr_to_gray(img))
        ts = float(frame_set.timestamp)
        prior = None
        if self._filt is not None:
            if not hasattr(self, "_samples"):
                self._samples = {}
            d = getattr(frame_set, "sensor_data", None)
            get = (d.get if isinstance(d, dict) else (lambda k: getattr(d, k, None))) if d is not None else None
            gy = None if get is None else get("gyroscope")
            sample = None if gy is None else (np.asarray(gy, dtype=np.float64).reshape(3),
                                              None if get("accelerometer") is None
                                              else np.asarray(get("accelerometer"), dtype=np.float64).reshape(3))
            smp = self._imu_priors(ts, sample)
            if self._filt.ready:
                prior = lagged_priors(self._filt, self._pending, [smp])[0]
        outs = [trk.step(imgs[2 * q], imgs[2 * q + 1], prior=prior if q == 0 else None)
                for q, trk in enumerate(self._trackers)]
        self.results.append(outs)
        g = self._g
        if self._filt is not None:
            self._pending.append((g, [(g, outs[0], prior)], [self._samples[g]]))
        self._prev_ts = ts
        if len(self._pairs) == 1:
            o = outs[0]
            status, raw = int(o["status"]), o["world_T_cam"]
            bt = self._E[0]
            cov = o["cov"] if status == 0 else np.zeros((6, 6))
            body = bt @ raw @ inv_rigid(bt)
            if self._ba is not None:
                self._ba.step(o)
                body = bt @ self._ba_correction(g, raw) @ inv_rigid(bt)
            if self._loop is not None:
                if status == 0 and g % self._config.loop_kf_interval == 0:
                    cfg = self._config
                    land = keyframe_landmarks(o["cur"]["left"], o["cur"]["disp"], self._intr)
                    land["feat"] = o["cur"]["left"]
                    self._db[len(self._loop.frames) % cfg.loop_max_keyframes] = land
                raw_c = inv_rigid(bt) @ body @ bt
                body = bt @ self._loop.step(g, status, raw_c) @ inv_rigid(bt)
        else:   # the rig's body motion from every pair, chained (numpy_imu.run_rig_sequence's rule)
            if g == 0:
                res = {"status": 2, "T": np.eye(4), "cov": np.zeros((6, 6))}
            else:
                items = [{"status": x["status"], "T": x["T"], "corr": x.get("corr"),
                          "intr": (d["fx"], d["fy"], d["cx"], d["cy"])} for x, d in zip(outs, self._rect_d)]
                res = rig_pose(items, self._E, self._config)
            if res["status"] == 0:
                self._T_body = self._T_body @ inv_rigid(res["T"])
            status, body, cov = int(res["status"]), self._T_body.copy(), res["cov"] if res["status"] == 0 else np.zeros((6, 6))
        self._g += 1
        if status == 1:
            self._state, self._latest = self._TS.LOST, None
            return None
        from thor_slam_amd.calib import confidence_from_covariance
        from thor_slam_amd.slam.interface import SlamPose

        self._state = self._TS.TRACKING if status == 0 else self._TS.INITIALIZING
        self._latest = SlamPose(position=body[:3, 3].copy(), rotation=_quat(body[:3, :3]), timestamp=ts,
                                tracking_state=self._state,
                                confidence=confidence_from_covariance(cov) if status == 0 else 1.0, covariance=cov)
        return self._latest

    def _ba_correction(self, g: int, raw: np.ndarray) -> np.ndarray:
        """W_ba(kf) inv(W_fe(kf)) W_fe(g) with kf the newest window keyframe at or before g."""
        cfg, w = self._config, self._ba.win
        if g % cfg.ba_kf_interval == 0:
            self._fe_at[g] = raw.copy()
        live = {int(f): inv_rigid(w.T_cw[s]) for s, f in enumerate(w.frames) if f >= 0}
        if not live:
            return raw
        kf = max([f for f in live if f <= g], default=min(live))
        return live[kf] @ inv_rigid(self._fe_at[kf]) @ raw

    def get_tracking_state(self):
        return self._state

    def get_map(self):
        from thor_slam_amd.slam.interface import SlamMap, SlamPose

        kfs = []
        if self._loop is not None:
            bt = self._E[0]
            for g, T in zip(self._loop.frames, self._loop.T):
                body = bt @ T @ inv_rigid(bt)
                kfs.append(SlamPose(position=body[:3, 3].copy(), rotation=_quat(body[:3, :3]), timestamp=float(g),
                                    tracking_state=self._TS.TRACKING, confidence=1.0))
        return SlamMap(keyframe_poses=kfs)

    def reset(self) -> None:
        self._reset_state()
        if hasattr(self, "_samples"):
            self._samples = {}
        self._state = self._TS.INITIALIZING
        self.frame_count = 0

    def shutdown(self) -> None:
        self._trackers = []
        self._state = self._TS.NOT_INITIALIZED

    def save_map(self, path: str) -> bool:
        return False

    def load_map(self, path: str) -> bool:
        return False

    def relocalize(self) -> bool:
        return False
