"""``HipSlamEngine`` — the MI355X back end behind the reference ``SlamEngine`` interface.

Drop-in replacement for ``IsaacRosAdapter`` (``thor_slam/slam/adapters/isaac_ros.py:59-458``):

* construction ``HipSlamEngine(num_cameras=N)`` like ``IsaacRosAdapter(num_cameras)``
  (``scripts/run_slam.py:299``);
* ``initialize`` extracts the flat camera list exactly like ``_extract_cameras`` (isaac_ros.py:
  138-157), pairs ``cam_idx`` 0/1 of a source into stereo pairs (the rule of isaac_ros.py:393),
  builds the rectification that cuVSLAM performs internally (``rectified_images:=false``,
  Makefile:80) and allocates the device workspace;
* ``process_frames`` raises ``RuntimeError("Not initialized")`` before ``initialize``
  (isaac_ros.py:329-330), skips cameras whose source or ``cam_idx`` is absent (:337-341),
  converts 3-channel BGR frames to gray, and returns the newest pose (``None`` when tracking is
  lost, per interface.py:197-199);
* ``reset`` -> INITIALIZING (:438-442), ``shutdown`` -> NOT_INITIALIZED (:444-450).

Poses are world_T_base (base_link of the rig; world = base_link at the first frame), obtained by
conjugating the tracked rectified-left-camera motion with base_T_camera from the calibration.
With local BA on (``ba_window > 0``, SURVEY.md §8a A8, one stereo pair) a frame's pose is the
front-end pose carried by the correction of the newest keyframe at or before it that is still in
the window, ``W_ba(kf) inv(W_fe(kf)) W_fe(g)`` (the oldest window keyframe's when the batch has
already evicted it), and ``get_map`` returns the keyframes (BA estimates) and the window's
landmarks.  With several pairs the keyframes of all pairs form ONE window of body poses (the
rig-level solve, ``handle.ba_read(n_pairs)``; each pair keeps its landmarks, ``ba_read(p)``): the
published pose is the rig's front end carried by the body correction ``B_ba(kf) inv(B_fe(kf))``,
and ``get_map`` returns the body keyframes and every pair's landmarks.
With ``dense_map`` (RGB-D input) every batch's depth of pair 0 is integrated into a dense TSDF
volume on the device with the batch's tracked poses (nvblox's role in the reference pipeline,
``scripts/run_pipeline.py:218-256``); ``get_dense_map`` returns it.
With ``HipSlamConfig(devices=[d0, d1, ...])`` the rig is sharded one camera stream per GPU from
this one process (cuVSLAM's multicam mode, launch/thor_visual_slam.launch.py:49,81):
one handle per device, driven by the library as one sharded rig (``tslam_group_*``: an RCCL clique
over the devices, or device copies with ``shard_transport="copy"``).  It has the one-device engine's
features: batches of any length (a short last batch at ``flush``), asynchronous submission (the
driver's pinned result slots, polled like ``tslam_submit_host``'s), and — through the driver's
state gather to rank 0 (``TSLAM_SHARD_GATHER``) — local BA (solved by rank 0), loop closure and
relocalisation on rank 0's handle; the published poses are bit-identical to the one-device engine's.
``confidence`` follows isaac_ros.py:312.  With ``batch_size > 1`` frames are staged and the
batch runs on the GPU when full (or on ``flush``).  Submission is asynchronous
(``tslam_submit_host``: pinned double-buffered staging, the batch's H2D copy and kernels on the
handle's own streams, results copied back into pinned slots) and completed batches are
published by non-blocking polls, so the host prepares batch s+1 while the device runs batch s;
the returned pose is the latest completed one, as the reference allows (its pose lags the
published frame, isaac_ros.py:429-430).  Local BA, loop closure and the dense map read device
state per batch, so with those on every batch is waited for before the next one is staged.
"""

from __future__ import annotations

import collections
import logging
import math
import threading

import numpy as np
from scipy.spatial.transform import Rotation

from .._lib import POSE_INIT, POSE_LOST, POSE_OK, Handle, HandleGroup, SingularSystemError
from ..calib import (StereoRectification, confidence_from_covariance, extract_cameras, rgbd_pairs, rgbd_undistort,
                     stereo_pairs, stereo_rectify)
from ..camera.rig import RigCalibration
from ..loop import span_edges
from ..camera.types import SynchronizedFrameSet
from ..imu import ImuNoise, ImuPropagator, vision_only
from ..params import HipSlamConfig
from ..rgbd import pack_rgbd
from .interface import CameraConfig, MapPoint, SlamConfig, SlamEngine, SlamMap, SlamPose, TrackingState

logger = logging.getLogger(__name__)


def bgr_to_gray(img: np.ndarray) -> np.ndarray:
    """8-bit BGR -> gray with the fixed-point BT.601 weights (R 4899, G 9617, B 1868) / 2^14."""
    if img.ndim == 2:
        return img
    b = img[..., 0].astype(np.int32)
    g = img[..., 1].astype(np.int32)
    r = img[..., 2].astype(np.int32)
    return ((r * 4899 + g * 9617 + b * 1868 + 8192) >> 14).astype(np.uint8)


def adjoint(t: np.ndarray) -> np.ndarray:
    """SE(3) adjoint of a rigid 4x4 in the solver's (rho, omega) twist order: a left perturbation
    exp(xi) of a pose P becomes exp(Ad_T xi) of T P T^-1, so cov' = Ad cov Ad^T with
    Ad = [[R, [t]x R], [0, R]]."""
    r, tv = t[:3, :3], t[:3, 3]
    tx = np.array([[0.0, -tv[2], tv[1]], [tv[2], 0.0, -tv[0]], [-tv[1], tv[0], 0.0]])
    ad = np.zeros((6, 6))
    ad[:3, :3] = ad[3:, 3:] = r
    ad[:3, 3:] = tx @ r
    return ad


def _quat_xyzw(m: np.ndarray) -> np.ndarray:
    """(x, y, z, w) of a rotation matrix — scipy's ``Rotation.from_matrix(m).as_quat()`` formula
    (the largest of the diagonal and the trace picks the branch; bit-identical on orthonormal input,
    checked in tests/test_boundary.py) in plain floats: the per-frame publish path avoids scipy's
    ~30-60 us of validation per call."""
    m00, m01, m02 = float(m[0, 0]), float(m[0, 1]), float(m[0, 2])
    m10, m11, m12 = float(m[1, 0]), float(m[1, 1]), float(m[1, 2])
    m20, m21, m22 = float(m[2, 0]), float(m[2, 1]), float(m[2, 2])
    tr = m00 + m11 + m22
    d = (m00, m11, m22, tr)
    c = max(range(4), key=d.__getitem__)
    if c == 3:
        q = [m21 - m12, m02 - m20, m10 - m01, 1.0 + tr]
    else:
        M = ((m00, m01, m02), (m10, m11, m12), (m20, m21, m22))
        i = c
        j = (i + 1) % 3
        k = (j + 1) % 3
        q = [0.0, 0.0, 0.0, 0.0]
        q[i] = 1.0 - tr + 2.0 * M[i][i]
        q[j] = M[j][i] + M[i][j]
        q[k] = M[k][i] + M[i][k]
        q[3] = M[k][j] - M[j][k]
    n = math.sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3])
    return np.array([q[0] / n, q[1] / n, q[2] / n, q[3] / n])


def _invert(t: np.ndarray) -> np.ndarray:
    out = np.eye(4)
    out[:3, :3] = t[:3, :3].T
    out[:3, 3] = -t[:3, :3].T @ t[:3, 3]
    return out


class _LoopGraph:
    """Host side of loop closure: keyframe nodes (rect-left world_T_cam), edges, and the
    correction applied to poses after the last solve (corrected = corr @ raw)."""

    def __init__(self) -> None:
        self.frames: list[int] = []
        self.stamps: list[float] = []
        self.raw: list[np.ndarray] = []     # pose at insertion, before loop correction
        self.T: list[np.ndarray] = []       # current (optimised) node poses
        self.edges: list[tuple[int, int]] = []
        self.meas: list[np.ndarray] = []
        self.info: list[np.ndarray] = []
        self.loops: list[tuple[int, int, int]] = []
        self.pairs: list[tuple[int, int]] = []     # per loop: (pair of the older entry, verifying pair)
        self.corr = np.eye(4)
        self.cost = 0.0
        self.full = False

    @staticmethod
    def information(cfg) -> np.ndarray:
        return np.diag([1.0 / cfg.pg_sigma_t ** 2] * 3 + [1.0 / cfg.pg_sigma_r ** 2] * 3)


class _AsyncLoop(_LoopGraph):
    """Loop closure without host waits (one device, ``tslam_loop_auto``): the policy of
    ``oracle/numpy_loop.py`` ``LoopPolicy`` on the device's loop jobs.  The submit path stores every
    keyframe in the database in stream order; a tracked keyframe becomes a node whose search
    (signature votes -> verification -> span solve) runs as jobs on the handle's loop stream while
    tracking goes on; items progress at every call without waiting and complete, oldest first, at
    the latest when their due frame (keyframe + ``loop_latency``) is published — so the published
    poses are a function of the data alone, whatever the timing."""

    MAX_JOBS = 48   # of the library's 64 unreturned job slots

    def __init__(self, handle: Handle, cfg: HipSlamConfig, n_pairs: int, rect0_T_rect: list) -> None:
        super().__init__()
        self.h, self.cfg, self.P = handle, cfg, n_pairs
        self.m = rect0_T_rect
        self.info_m = self.information(cfg)
        self.odo: list = []
        self.items: collections.deque = collections.deque()
        self.jobs = 0   # submitted, not yet returned
        self._busy = False
        self.last_loop: int | None = None   # node of the last closed loop (loop_cooldown)
        self.trace: dict | None = None   # set to {} to record every job's inputs and results (tests)
        self.failures: list = []
        self.rejected: list = []   # (keyframe of c, g) of loops whose span solve was rejected
        # relocalisation after a LOST run (LoopPolicy.observe / _relocate)
        self.lost_run = 0
        self.reloc = False          # RELOCALIZING
        self.anchor_end = 0         # candidates of the episode: nodes < anchor_end
        self.seg_start = 0          # first node of the unanchored segment
        self.relocs: list = []      # (keyframe of c, g, inliers)
        self.last_due = -1

    def observe(self, g: int, status: int) -> None:
        """oracle LoopPolicy.observe: the LOST-run bookkeeping of frame g."""
        if status == POSE_LOST:
            self.lost_run += 1
            after = self.cfg.reloc_after_lost
            if after > 0 and self.lost_run == after and self.frames:
                if not self.reloc:
                    self.reloc = True
                    self.anchor_end = len(self.frames)
                self.seg_start = len(self.frames)
        else:
            self.lost_run = 0

    # -- oracle LoopPolicy._node: node idx = database position idx (tslam_loop_auto) ----------
    def node(self, g: int, raw: np.ndarray, ts: float) -> None:
        idx = len(self.frames)
        if idx == 0 or (self.reloc and idx == self.seg_start):   # the first node of a segment
            T, Z = self.corr @ raw, None
        else:
            Z = _invert(self.raw[-1]) @ raw
            T = self.T[-1] @ Z
            self.edges.append((idx - 1, idx))
            self.meas.append(Z)
            self.info.append(self.info_m)
        self.frames.append(g)
        self.stamps.append(ts)
        self.raw.append(raw.copy())
        self.T.append(T)
        self.odo.append(Z)
        cfg = self.cfg
        kind = "reloc" if self.reloc else "loop"
        lo, hi = self._reloc_window(idx) if self.reloc else self._window(idx)
        due = max(g + (cfg.reloc_latency if self.reloc else cfg.loop_latency), self.last_due)
        self.last_due = due
        it = {"idx": idx, "g": g, "due": due, "lo": lo, "n_kf": hi - lo + 1, "kind": kind,
              "stage": "new" if hi >= lo else "done"}
        self.items.append(it)
        self._progress(it, False, len(self.items) == 1)

    def _window(self, idx: int) -> tuple[int, int]:   # oracle numpy_loop.candidate_window
        cfg = self.cfg
        margin = (cfg.loop_latency + 2 * cfg.batch_size - 1) // cfg.loop_kf_interval + 1
        return max(0, idx - cfg.loop_max_keyframes + margin), idx - cfg.loop_min_gap

    def _reloc_window(self, idx: int) -> tuple[int, int]:   # oracle LoopPolicy.reloc_window
        cfg = self.cfg
        margin = (cfg.loop_latency + 2 * cfg.batch_size - 1) // cfg.loop_kf_interval + 1
        return max(0, idx - cfg.loop_max_keyframes + margin), self.anchor_end - 1

    def _entry(self, pos: int, p: int) -> int:
        return (pos % self.cfg.loop_max_keyframes) * self.P + p

    def _result(self, job, block: bool):
        # jobs finish in submission order on the loop stream: once one is still running, a later
        # one is too, so this pass polls no further (each poll is an event query)
        if not block and self._busy:
            return None
        try:
            r = job.result(block)
        except RuntimeError:   # a failed job is returned too (its slot is free): count it out
            self.jobs -= 1
            raise
        if r is not None:
            self.jobs -= 1
        elif not block:
            self._busy = True
        return r

    # -- progress without waiting; `block`: complete it (its due frame is being published) --------
    def advance(self, until: int | None = None) -> None:
        first = True
        self._busy = False
        for it in list(self.items):
            must = until is not None and it["due"] <= until
            self._progress(it, must, first)
            if it["stage"] != "done":
                if must:
                    raise RuntimeError("loop closure: a due item did not complete")
                first = False
                continue
            if first:
                self.items.popleft()

    def _progress(self, it: dict, block: bool, head: bool) -> None:
        cfg, P, h = self.cfg, self.P, self.h
        if it["stage"] == "new":
            if self.jobs + P > self.MAX_JOBS and not block:
                return
            it["votes"] = [h.loop_job_vote(self._entry(it["idx"], q), it["lo"], it["n_kf"]) for q in range(P)]
            self.jobs += P
            it["stage"] = "vote"
        if it["stage"] == "vote":
            got = it.setdefault("got", [None] * P)
            for q, job in enumerate(it["votes"]):
                if got[q] is None:
                    try:
                        got[q] = self._result(job, block)
                    except RuntimeError:   # a failed job (a device error): the item ends here (its
                        it["stage"] = "done"  # other vote jobs stay counted: their slots are unreturned
                        raise
            if any(v is None for v in got):
                return
            if self.trace is not None:
                for q, v in enumerate(got):
                    self.trace[("vote", it["idx"], q)] = (it["lo"], it["n_kf"], v.copy())
            # oracle numpy_loop.best_vote: most votes; ties to the lower query pair, then the newest
            # position (the smallest span), then the lower pair
            best, q, j = -1, 0, 0
            for qq in range(P):
                v = got[qq].reshape(-1, P)
                r = int(np.argmax(v[::-1].reshape(-1)))
                jj = (v.shape[0] - 1 - r // P) * P + r % P
                if int(got[qq][jj]) > best:
                    best, q, j = int(got[qq][jj]), qq, jj
            if best < cfg.loop_min_votes:
                it["stage"] = "done"
                return
            c, pc = it["lo"] + j // P, j % P
            it.update(q=q, c=c, pc=pc, stage="verify")
            it["job"] = h.loop_job_verify(it["g"], self._entry(it["idx"], q), self._entry(c, pc), pair=q)
            self.jobs += 1
        if it["stage"] == "verify":
            try:
                ver = self._result(it["job"], block)
            except RuntimeError:   # a failed job (a device error): the item ends here
                it["stage"] = "done"
                raise
            if ver is None:
                return
            if self.trace is not None:
                self.trace[("verify", it["idx"])] = (it["q"], it["c"], it["pc"], ver)
            if int(ver["stats"][0]) != POSE_OK or int(ver["stats"][2]) < cfg.loop_min_inliers:
                it["stage"] = "done"
                return
            it.update(ver=ver, stage="verified")
        if it["kind"] == "reloc":
            if it["stage"] == "verified" and block:   # applied at the due frame (LoopPolicy._relocate)
                self._relocate(it)
                it["stage"] = "done"
            return
        if it["stage"] == "verified" and head:
            # the span solve starts once every older item is applied, so its inputs (the span's
            # poses and edges, with this loop's edge) are what they are at the due frame
            a, idx, q, pc = it["c"], it["idx"], it["q"], it["pc"]
            if self.last_loop is not None and idx - self.last_loop <= cfg.loop_cooldown:
                it["stage"] = "done"   # within the cooldown of the last closed loop
                return
            it["last_loop"] = self.last_loop   # restored when the span solve is rejected
            self.last_loop = idx
            ver = it["ver"]
            it["edge"] = (a, idx, self.m[pc] @ _invert(ver["T"]) @ _invert(self.m[q]))
            edges = self.edges + [(a, idx)]
            meas = self.meas + [it["edge"][2]]
            sel = span_edges(edges, a, idx)
            args = (np.stack(self.T[a:idx + 1]), np.array([edges[e] for e in sel]) - a, np.stack([meas[e] for e in sel]),
                    np.stack([self.info_m] * len(sel)))
            it["job"] = h.loop_job_pose_graph(*args, cfg.pg_iters)
            it["args"] = args
            self.jobs += 1
            it.update(a=a, stage="solve")
        if it["stage"] == "solve":
            try:
                sol = self._result(it["job"], block)
            except SingularSystemError as exc:
                # LoopPolicy's rejection: the span's normal matrix is not positive definite, so the
                # loop is dropped (no edge, no correction, the cooldown unchanged) and tracking goes
                # on — process_frames keeps the reference's contract (interface.py:192-200)
                self.failures.append({"idx": it["idx"], "g": it["g"], "args": it["args"], "ver": it["ver"],
                                      "q": it["q"], "c": it["c"], "pc": it["pc"], "error": str(exc)})
                self.rejected.append((self.frames[it["a"]], it["g"]))
                self.last_loop = it["last_loop"]
                if self.trace is not None:
                    self.trace[("solve", it["idx"])] = (it["args"], None)
                it["stage"] = "done"
                logger.warning("loop closure: keyframe %d -> %d rejected (%s)", self.frames[it["a"]], it["g"], exc)
                return
            if sol is None:
                return
            it.update(sol=sol, stage="solved")
        if it["stage"] == "solved" and block:   # applied at the due frame, as LoopPolicy does
            a, idx, sol, ver = it["a"], it["idx"], it["sol"], it["ver"]
            if self.trace is not None:
                self.trace[("solve", idx)] = (it["args"], sol)
            self.edges.append((a, idx))
            self.meas.append(it["edge"][2])
            self.info.append(self.info_m)
            self.loops.append((self.frames[a], it["g"], int(ver["stats"][2])))
            self.pairs.append((it["pc"], it["q"]))
            self.T[a:idx + 1] = list(sol["T"])
            for i in range(idx + 1, len(self.T)):
                if self.odo[i] is None:   # a segment break: the nodes after it are anchored otherwise
                    break
                self.T[i] = self.T[i - 1] @ self.odo[i]
            self.corr = self.T[-1] @ _invert(self.raw[-1])
            self.cost = sol["cost"]
            it["stage"] = "done"
            logger.info("loop closure: keyframe %d -> %d (%d inliers), span of %d nodes, cost %.3g",
                        self.frames[a], it["g"], int(it["ver"]["stats"][2]), idx - a + 1, sol["cost"])


    def _relocate(self, it: dict) -> None:
        """oracle LoopPolicy._relocate, from the item's verified candidate: the unanchored
        segment moves rigidly onto the candidate keyframe's pose and tracking resumes."""
        idx, c, q, pc, ver = it["idx"], it["c"], it["q"], it["pc"], it["ver"]
        if not self.reloc or idx < self.seg_start:
            return
        Z = self.m[pc] @ _invert(ver["T"]) @ _invert(self.m[q])
        D = self.T[c] @ Z @ _invert(self.T[idx])
        for i in range(self.seg_start, len(self.T)):
            self.T[i] = D @ self.T[i]
        self.edges.append((c, idx))
        self.meas.append(Z)
        self.info.append(self.info_m)
        self.corr = D @ self.corr
        self.relocs.append((self.frames[c], it["g"], int(ver["stats"][2])))
        self.reloc = False
        self.last_loop = idx
        logger.info("relocalised: keyframe %d against keyframe %d (%d inliers)", it["g"], self.frames[c],
                    int(ver["stats"][2]))


class HipSlamEngine(SlamEngine):
    """Stereo visual odometry front end (detect -> match -> pose) running on one MI355X."""

    def __init__(self, num_cameras: int = 2, config: HipSlamConfig | None = None, device: int = 0) -> None:
        self._num_cameras = num_cameras
        self._config = config or HipSlamConfig(num_cameras=num_cameras)
        self._device = device
        self._state = TrackingState.NOT_INITIALIZED
        self._cameras: list[CameraConfig] = []
        self._pairs: list[tuple[int, int]] = []
        self._rects: list[StereoRectification] = []
        self._handle: Handle | None = None
        self._base_T_rect: np.ndarray | None = None
        self._latest_pose: SlamPose | None = None
        self._pose_lock = threading.Lock()
        # the map state _publish grows (BA keyframes, landmarks, loop graph) against readers on other
        # threads (get_map / save_map while process_frames runs; the reference adapter's locks,
        # isaac_ros.py:82,314,429)
        self._map_lock = threading.RLock()
        self._frame_count = 0
        self._staged: list[tuple[np.ndarray, float]] = []
        self._staged_imu: list[tuple | None] = []    # (gyro, accel) per staged frame
        self._imu: ImuPropagator | None = None       # IMU filter (gyro bias; accelerometer leg with imu_accel)
        # submitted batches whose vision the IMU filter has not absorbed yet, in order: {"n": batch
        # number, "samples", "steps", "res": the absorb inputs once published} (no "samples": no data)
        self._imu_batches: list = []
        self._imu_seq = 0                            # batches submitted (numbers the entries)
        self._kf_imu: tuple | None = None             # gyro rotation since the last BA keyframe (R, var, first frame)
        self._kf_ine: tuple | None = None             # samples since the last BA keyframe (list, first frame, w_prev)
        self._prev_stamp: float | None = None      # timestamp of the last submitted frame (IMU dt)
        self._base_R_imu = np.eye(3)
        self._base_T_imu = np.eye(4)
        self._torch = None
        self._dev_images = None
        self._host_images = None
        self._keyframe_poses: list[SlamPose] = []
        self._fe_at: dict[int, np.ndarray] = {}      # front-end rect world_T_cam of BA keyframes
        self._kf_final: dict[int, np.ndarray] = {}   # last BA estimate (rect world_T_cam) per keyframe
        self._kf_stamp: dict[int, float] = {}
        self._ba_window: dict | None = None
        self._ba_pairs: list[dict] = []
        self._map_points: dict[int, tuple] = {}   # global landmark id -> (xyz rect-0 frame, desc, observations)
        self._map_offset = np.eye(4)              # map world <- session world, set by relocalize()
        self._map_loaded = False
        self._loop: _LoopGraph | None = None     # set up by initialize() when loop closure is on
        self._in_flight = 0                       # batches submitted, not yet published
        self._shard: dict | None = None           # sharded rig (config.devices): handles, group, inputs

    # ------------------------------------------------------------------------------------------
    def initialize(self, calibration: RigCalibration, config: SlamConfig | None = None) -> None:
        if isinstance(config, HipSlamConfig):
            self._config = config
        cfg = self._config
        try:
            cfg.validate()
            self._cameras = extract_cameras(calibration, self._num_cameras)
            if len(self._cameras) < self._num_cameras:
                logger.warning("Calibration has %d cameras, expected %d", len(self._cameras), self._num_cameras)
            if cfg.rgbd:   # per source: colour camera (cam_idx 0) + aligned depth (cam_idx 1)
                self._pairs = rgbd_pairs(self._cameras)
                if not self._pairs:
                    raise RuntimeError("HipSlamEngine(rgbd) needs an RGB-D source (colour cam_idx 0, depth cam_idx 1)")
                self._rects = [rgbd_undistort(self._cameras[l]) for l, _ in self._pairs]
            else:
                self._pairs = stereo_pairs(self._cameras)
                if not self._pairs:
                    raise RuntimeError("HipSlamEngine needs at least one stereo source (cam_idx 0 and 1)")
                self._rects = [stereo_rectify(self._cameras[l], self._cameras[r]) for l, r in self._pairs]
            import torch  # PyTorch is the device-memory / stream plumbing only

            if not torch.cuda.is_available():
                raise RuntimeError("no ROCm device visible: the MI355X back end has no CPU fallback")
            self._torch = torch
            rect0 = self._rects[0]
            if cfg.rgbd:   # one [BGR | u16 depth] record of 5*H*W bytes per camera
                shape = (cfg.batch_size, len(self._pairs), 5 * rect0.height * rect0.width)
            else:
                shape = (cfg.batch_size, 2 * len(self._pairs), rect0.height, rect0.width)
            if cfg.devices:
                self._init_shard(shape)
            else:
                self._handle = Handle(self._rects, cfg, max_batch=cfg.batch_size, device=self._device)
                self._dev_images = torch.empty(shape, dtype=torch.uint8, device=f"cuda:{self._device}")
                self._host_images = torch.empty(shape, dtype=torch.uint8).pin_memory()
            self._base_T_rects = [self._cameras[l].extrinsics.to_4x4_matrix() @ r.left_optical_T_rect()
                                  for (l, _), r in zip(self._pairs, self._rects)]
            self._base_T_rect = self._base_T_rects[0]
            self._bt_inv = _invert(self._base_T_rect)        # cached for the per-frame publish path
            self._prior_moves = None
            self._bt_ad = adjoint(self._base_T_rect)
            imu = getattr(calibration, "imu_extrinsics", None)   # world(base)_T_imu, RDF-converted by the caller
            base_T_imu = imu.to_4x4_matrix() if imu is not None else np.eye(4)
            self._base_R_imu = base_T_imu[:3, :3]
            self._base_T_imu = base_T_imu
            self._imu = None
            # the reference fuses the IMU whenever it has one (enable_imu_fusion:=true, Makefile:81)
            fusion = cfg.imu_fusion if cfg.imu_fusion is not None else imu is not None
            if fusion:
                accel = cfg.imu_accel if cfg.imu_accel is not None else True
                noise = ImuNoise(cfg.gyroscope_noise_density, cfg.gyroscope_random_walk, cfg.accelerometer_noise_density,
                                 cfg.accelerometer_random_walk, cfg.imu_rot_floor, cfg.imu_trans_floor,
                                 ba0_sigma=cfg.imu_accel_bias_sigma, bg0_sigma=cfg.imu_gyro_bias_sigma,
                                 vis_rot_floor=cfg.imu_vis_rot_floor)
                rect_T_imu = _invert(self._base_T_rect) @ base_T_imu   # the IMU in pair 0's rectified-left camera
                self._imu = ImuPropagator(rect_T_imu[:3, :3], noise, lever=rect_T_imu[:3, 3], accel=accel)
            if len(self._pairs) > 1 and self._shard is None:   # the rig's body motion, on the device from all pairs
                self._handle.set_rig(self._base_T_rects)
            if cfg.dense_map:
                if cfg.dense_color:
                    self._handle.tsdf_color(True)
                self._handle.tsdf_init(cfg.tsdf_origin, cfg.tsdf_dims, cfg.voxel_size,
                                       cfg.tsdf_integrator_truncation_distance_vox,
                                       cfg.tsdf_integrator_max_integration_distance_m, cfg.tsdf_max_weight)
            self._loop = None
            if cfg.enable_loop_closure and cfg.devices and cfg.rgbd:
                # rank 0's ring holds only its own cameras' features (no state gather): no rig-wide
                # place recognition
                logger.warning("loop closure is off on a camera-sharded RGB-D rig")
            elif cfg.enable_loop_closure:
                # place recognition over every pair's camera (P database entries per keyframe,
                # keyframe-major) and verification on the pair that voted best; the keyframe nodes
                # are pair 0's rectified-left poses (on a multi-pair rig taken from the rig's body
                # poses, k_rig_pose), and the pose-graph correction moves the body poses
                cap = cfg.loop_max_keyframes * len(self._pairs)
                if cap > 1 << 16:
                    raise ValueError(f"loop_max_keyframes * pairs = {cap} exceeds the 65536-entry database")
                self._handle.loop_init(cap, cfg.loop_signature)
                if self._shard is None:   # the submit path stores the keyframes; searches run as loop jobs
                    self._handle.loop_auto(cfg.loop_kf_interval)
                    m = [_invert(self._base_T_rects[0]) @ e for e in self._base_T_rects]
                    self._loop = _AsyncLoop(self._handle, cfg, len(self._pairs), m)
                else:
                    self._loop = _LoopGraph()
        except RuntimeError:
            raise
        except Exception as exc:  # per interface.py:187-188
            raise RuntimeError(f"HipSlamEngine initialisation failed: {exc}") from exc
        self._state = TrackingState.INITIALIZING
        logger.info("Initialized HIP SLAM with %d cameras, %d stereo pair(s)", len(self._cameras), len(self._pairs))

    def _init_shard(self, shape: tuple) -> None:
        """One handle per device (the whole rig on each, rank r owning cameras [r*S, (r+1)*S)) and
        the library's group driver over them, with the state gather to rank 0 (local BA, loop
        closure and relocalisation run on rank 0's handle) and pinned result slots (asynchronous
        polling); pinned staging + device input per rank and batch parity."""
        torch, cfg = self._torch, self._config
        devs = [int(d) for d in cfg.devices]
        world = len(devs)
        n_cams = shape[1]
        if n_cams % world:
            raise RuntimeError(f"{n_cams} cameras do not split over {world} devices")
        handles = []
        for d in devs:
            h = Handle(self._rects, cfg, max_batch=cfg.batch_size, device=d)
            if len(self._rects) > 1:
                h.set_rig([self._cameras[l].extrinsics.to_4x4_matrix() @ r.left_optical_T_rect()
                           for (l, _), r in zip(self._pairs, self._rects)])
            handles.append(h)
        group = HandleGroup(handles, cfg.shard_transport)
        # results through the slots; the state gather (rank 0's ring as the one-handle path's) is the
        # stereo rig's: a camera-sharded RGB-D rig moves pair blocks and keeps no rig-wide ring
        handles[0].shard_options(gather=not cfg.rgbd, results=True, pipeline=True)
        S = n_cams // world
        part = (cfg.batch_size, S) + tuple(shape[2:])
        self._shard = {"handles": handles, "group": group, "world": world, "S": S, "devices": devs, "batches": 0,
                       "stamps": collections.deque(),
                       "dev": [[torch.empty(part, dtype=torch.uint8, device=f"cuda:{d}") for _ in range(2)] for d in devs],
                       "host": [[torch.empty(part, dtype=torch.uint8).pin_memory() for _ in range(2)] for _ in devs],
                       "h2d": [[None, None] for _ in devs]}
        self._handle = handles[0]   # every rank ends a batch with the whole rig's poses; rank 0 has the rest

    def _submit_sharded(self) -> None:
        """The staged frames (any count up to batch_size) through the group driver, rank r getting
        its cameras' slice; the batch's results are polled from rank 0's pinned slots."""
        sh, torch = self._shard, self._torch
        n = len(self._staged)
        batch, imus = self._staged, self._staged_imu
        stamps = [ts for _, ts in batch]
        if self._imu is not None:
            self._set_imu_prior(stamps, imus)
        k = sh["batches"] & 1
        S, ptrs, streams = sh["S"], [], []
        for r, d in enumerate(sh["devices"]):
            if sh["h2d"][r][k] is not None:   # the pinned buffer of this parity: batch s-2's copy is done
                sh["h2d"][r][k].synchronize()
            host = sh["host"][r][k].numpy()
            for i, (imgs, _) in enumerate(batch):
                host[i] = imgs[r * S:(r + 1) * S]
            stream = torch.cuda.current_stream(d)
            # the device input of this parity: the driver made this stream wait for batch s-2
            sh["dev"][r][k][:n].copy_(sh["host"][r][k][:n], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(stream)
            sh["h2d"][r][k] = ev
            ptrs.append(sh["dev"][r][k].data_ptr())
            streams.append(stream.cuda_stream)
        if self._in_flight >= 2:   # rank 0 keeps two batches' results: publish the older first
            self._drain(block=True, limit=1)
        sh["group"].submit(ptrs, n, streams)
        sh["stamps"].append(stamps)   # the driver's result slots carry frame indices, not timestamps
        sh["batches"] += 1
        self._in_flight += 1
        self._staged, self._staged_imu = [], []
        self._prev_stamp = stamps[-1]
        if not self._async:
            self._drain(block=True)
        if self._config.dense_map:
            # camera-sharded RGB-D: pair 0 is rank 0's first camera, and rank 0 ends the batch with
            # every pair's chained poses (the pose records' all-gather), so the volume lives on rank
            # 0 and integrates its own input with the device poses — no extra exchange (the batch
            # was waited for: the dense map keeps the engine synchronous)
            self._integrate_depth(sh["dev"][0][k].data_ptr(), n, torch.cuda.current_stream(sh["devices"][0]).cuda_stream,
                                  cams_per_frame=S)

    # ------------------------------------------------------------------------------------------
    def _frame_images(self, frame_set: SynchronizedFrameSet, out: np.ndarray | None = None) -> np.ndarray | None:
        """The frame's input record ([2P][H][W] gray stereo, or [P][5HW] RGB-D), written into
        ``out`` (one flat row of the library's pinned staging, tslam_host_stage) when given — the
        batch then needs no stacking or staging copy — else stacked into a new array.  None when a
        camera of the rig is missing from the set."""
        imgs = []
        if self._config.rgbd:
            for c, d in self._pairs:
                cam = self._cameras[c]
                fs = frame_set.frame_sets.get(cam.source_name)
                if fs is None or max(cam.cam_idx, self._cameras[d].cam_idx) >= len(fs.frames):
                    return None
                bgr = np.asarray(fs.frames[cam.cam_idx].image)
                depth = np.asarray(fs.frames[self._cameras[d].cam_idx].image)
                if bgr.ndim == 2:
                    bgr = np.repeat(bgr[..., None], 3, axis=-1)
                if bgr.shape[:2] != (self._rects[0].height, self._rects[0].width) or depth.shape != bgr.shape[:2]:
                    raise ValueError(f"RGB-D camera {c}: colour {bgr.shape} / depth {depth.shape} do not match its calibration")
                imgs.append(pack_rgbd(bgr, depth.astype(np.uint16, copy=False)))
            return np.stack(imgs) if out is None else self._fill(out, imgs)
        for l, r in self._pairs:
            for gi in (l, r):
                cam = self._cameras[gi]
                fs = frame_set.frame_sets.get(cam.source_name)
                if fs is None or cam.cam_idx >= len(fs.frames):
                    return None
                img = bgr_to_gray(np.asarray(fs.frames[cam.cam_idx].image))
                if img.shape != (self._rects[0].height, self._rects[0].width):
                    raise ValueError(f"camera {gi} image shape {img.shape} does not match its calibration")
                imgs.append(img)
        return np.stack(imgs) if out is None else self._fill(out, imgs)

    @staticmethod
    def _fill(out: np.ndarray, imgs: list) -> np.ndarray:
        rows = out.reshape(len(imgs), -1)
        for i, im in enumerate(imgs):
            np.copyto(rows[i], np.asarray(im, dtype=np.uint8).reshape(-1))
        return out

    def process_frames(self, frame_set: SynchronizedFrameSet) -> SlamPose | None:
        if self._handle is None:
            raise RuntimeError("Not initialized")
        self._frame_count += 1
        if self._shard is None and not self._config.dense_map:   # straight into the pinned staging
            if not self._staged:
                self._stage = self._handle.host_stage()
            imgs = self._frame_images(frame_set, out=self._stage[len(self._staged)])
        else:
            imgs = self._frame_images(frame_set)
        if imgs is None:
            with self._pose_lock:
                return self._latest_pose
        self._staged.append((imgs, float(frame_set.timestamp)))
        self._staged_imu.append(self._imu_of(frame_set))
        if len(self._staged) >= self._config.batch_size:
            self._submit_staged()
        self._drain(block=False)
        if isinstance(self._loop, _AsyncLoop) and self._loop.items:
            with self._map_lock:
                self._loop.advance()   # submit / collect loop jobs without waiting
        with self._pose_lock:
            return self._latest_pose

    @property
    def _async(self) -> bool:
        """Batches may stay in flight across calls (nothing reads per-batch device state; an IMU
        filter that has seen no sample yet predicts nothing, so a rig whose calibration names an
        IMU that sends no data keeps the asynchronous path)."""
        cfg = self._config
        return (not cfg.sync and cfg.ba_window <= 0 and (self._loop is None or isinstance(self._loop, _AsyncLoop)) and not cfg.dense_map
                and (self._imu is None or not self._imu.ready or cfg.imu_prior_lag > 0))

    def _submit_staged(self) -> None:
        n = len(self._staged)
        if n == 0:
            return
        if self._shard is not None:
            self._submit_sharded()
            return
        stamps = [ts for _, ts in self._staged]
        if self._imu is not None:
            self._set_imu_prior(stamps, self._staged_imu)
        if self._config.dense_map:   # the TSDF reads the batch's depth records on the device
            torch = self._torch
            host = self._host_images.numpy()
            for k, (imgs, _) in enumerate(self._staged):
                host[k] = imgs
            stream = torch.cuda.current_stream(self._device)
            self._dev_images[:n].copy_(self._host_images[:n], non_blocking=True)
            self._handle.submit(self._dev_images.data_ptr(), n, stream.cuda_stream)
            self._integrate_depth(self._dev_images.data_ptr(), n, stream.cuda_stream)
            self._staged, self._staged_imu = [], []
            self._prev_stamp = stamps[-1]
            self._publish(self._read(n), stamps, self._handle.frames_done - n)
            return
        imgs = self._stage[:n]   # the frames were written there as they were staged (host_stage)
        if self._in_flight >= 2:   # the handle keeps two batches' results: publish the older first
            self._drain(block=True, limit=1)
        self._handle.submit_host(imgs, stamps)
        self._in_flight += 1
        self._staged, self._staged_imu = [], []
        self._prev_stamp = stamps[-1]
        if not self._async:
            self._drain(block=True)

    def _drain(self, block: bool, limit: int | None = None) -> None:
        """Publish completed batches in order (all in flight with ``block``; at most ``limit``)."""
        done = 0
        while self._in_flight > 0 and (limit is None or done < limit):
            res = self._handle.poll_batch(block=block)
            if res is None:
                return
            self._in_flight -= 1
            done += 1
            stamps = self._shard["stamps"].popleft() if self._shard is not None else list(res["timestamps"])
            self._publish(res, stamps, res["first_frame"])

    def flush(self) -> None:
        """Run the staged frames through the GPU pipeline and publish the poses of every batch
        submitted so far (waits for the device)."""
        if self._handle is None:
            return
        self._submit_staged()
        self._drain(block=True)

    def settle(self) -> None:
        """``flush`` and complete every pending loop-closure search now (oracle LoopPolicy.finish):
        the pose graph, ``loop_closures`` and the next published poses then include them."""
        self.flush()
        if isinstance(self._loop, _AsyncLoop):
            with self._map_lock:
                self._loop.advance(until=1 << 62)

    # -- IMU fusion -------------------------------------------------------
    @staticmethod
    def _imu_of(frame_set: SynchronizedFrameSet) -> tuple | None:
        """(gyroscope [rad/s], accelerometer [m/s^2] or None) in IMU axes of a synchronised set,
        from ``sensor_data`` (IMUData or a dict with "gyroscope" / "accelerometer"; rig.py:403-407)."""
        d = getattr(frame_set, "sensor_data", None)
        if d is None:
            return None
        get = d.get if isinstance(d, dict) else (lambda k: getattr(d, k, None))
        g, a = get("gyroscope"), get("accelerometer")
        if g is None:
            return None
        return (np.asarray(g, dtype=np.float64).reshape(3), None if a is None else np.asarray(a, dtype=np.float64).reshape(3))

    def _set_imu_prior(self, stamps: list[float], imus: list) -> None:
        """Per staged frame and pair: the motion predicted by the IMU filter (thor_slam_amd/imu.py)
        for pair 0's rectified-left camera over the frame interval — the bias-corrected gyro
        rotation with its weight and, with the accelerometer leg, the translation with its weight
        — moved into every other pair's camera through the rig, inv(E_p) E_0 T inv(E_0) E_p.  The
        samples are kept for the filter's update when the batch's results come back."""
        imu, prev = self._imu, self._prev_stamp
        seq = self._imu_seq
        self._imu_seq += 1
        self._imu_absorb_due(seq)
        if not imu.ready and all(s is None for s in imus):   # no IMU sample yet: nothing to predict,
            self._imu_batches.append({"n": seq, "res": None})  # and the batch may stay in flight
            return
        samples = []
        for ts, s in zip(stamps, imus):
            ok = s is not None and (s[1] is not None or not imu.accel)
            if ok and not imu.ready:
                imu.begin(s[1])            # this frame anchors the filter: no prior for it
                samples.append((None, None, None))
            elif ok and prev is not None and ts > prev:
                samples.append((ts - prev, s[0], s[1]))
            else:
                samples.append((None, None, None))
            prev = ts
        # the vision of the batches still pending (at most imu_prior_lag of them) is not in the
        # filter yet: the state coasts over their samples (oracle/numpy_imu.py lagged_priors)
        coast = [c for e in self._imu_batches if "samples" in e for c in e["samples"]]
        steps = imu.batch_priors(coast + samples)[len(coast):]
        self._ba_imu_factors(steps)
        self._ba_inertial_factors(steps, samples)
        P, n = len(self._pairs), len(stamps)
        rot = np.tile(np.eye(3), (n, P, 1, 1))
        trn = np.zeros((n, P, 3))
        wr, wt = np.zeros((n, P)), np.zeros((n, P))
        if getattr(self, "_prior_moves", None) is None:   # (inv(E_p) E_0, inv(E_0), E_p) per pair, once
            e0 = self._base_T_rects[0]
            self._prior_moves = [(_invert(ep) @ e0, _invert(e0), ep) for ep in self._base_T_rects]
        for k, st in enumerate(steps):
            if st is None:
                continue
            t0 = np.eye(4)
            t0[:3, :3], t0[:3, 3] = st.R_rel, st.t_rel
            for p, (a, ie0, ep) in enumerate(self._prior_moves):
                tp = t0 if p == 0 else a @ t0 @ ie0 @ ep   # the same products, in the same order, as before
                rot[k, p], trn[k, p] = tp[:3, :3], tp[:3, 3]
                wr[k, p], wt[k, p] = st.w_rot, st.w_trans
        self._set_motion_prior(rot, wr, trn, wt)
        self._imu_batches.append({"n": seq, "samples": samples, "steps": steps, "res": None})

    def _imu_absorb_due(self, seq: int) -> None:
        """Before batch ``seq``'s priors: the filter absorbs the vision of every batch numbered
        <= seq - 1 - imu_prior_lag (waiting for its results if needed), in order, and no other —
        whatever has already come back — so the priors are a function of the data alone."""
        lag = max(int(self._config.imu_prior_lag), 0)
        while self._imu_batches and self._imu_batches[0]["n"] <= seq - 1 - lag:
            while self._imu_batches[0]["res"] is None:
                if self._in_flight == 0:
                    raise RuntimeError("IMU filter: a batch to absorb was never published")
                self._drain(block=True, limit=1)
            e = self._imu_batches.pop(0)
            if "samples" in e:
                self._imu.absorb(e["samples"], *e["res"])

    def _ba_imu_factors(self, steps: list) -> None:
        """The local BA's IMU rotation factors (one stereo pair): the per-frame gyro rotations of
        the staged batch composed since the last keyframe; at each keyframe whose whole interval
        had IMU steps, the rotation from the previous keyframe's camera and the inverse of the
        summed rotation variances (1 / rad^2: the reprojection residuals have unit pixel weight)
        go to tslam_ba_imu_factor before the batch is submitted."""
        cfg = self._config
        if cfg.ba_window <= 0 or len(self._pairs) != 1:
            return
        if self._ine_on():   # the inertial records carry the gyro rotation (and the gyroscope bias)
            return
        g = self._handle.frames_done
        for k, st in enumerate(steps):
            gk = g + k
            if st is None or self._kf_imu is None:
                self._kf_imu = None if st is None else (st.R_rel.copy(), 1.0 / st.w_rot, gk)
            else:
                rot, var, start = self._kf_imu
                self._kf_imu = (st.R_rel @ rot, var + 1.0 / st.w_rot, start)
            if gk % cfg.ba_kf_interval == 0:
                acc = self._kf_imu
                if acc is not None and acc[2] == gk - cfg.ba_kf_interval + 1 and acc[1] > 0.0:
                    self._handle.ba_imu_factor(gk, acc[0], 1.0 / acc[1])
                self._kf_imu = (np.eye(3), 0.0, gk + 1)

    def _ine_on(self) -> bool:
        """The local BA takes tightly coupled inertial factors (accelerometer leg, filter started)."""
        imu = self._imu
        return (self._config.ba_window > 0 and bool(self._config.ba_inertial) and imu is not None and bool(imu.accel)
                and bool(imu.ready))

    def _ba_inertial_factors(self, steps: list, samples: list) -> None:
        """The local BA's tightly coupled inertial factors (accelerometer leg): the frame
        intervals' samples since the last BA keyframe are preintegrated with the filter's current
        biases (tslam_imu_preintegrate); at each keyframe whose whole interval had samples the
        record and the keyframe's predicted world velocity go to tslam_ba_inertial_factor, and the
        window gets the filter's gravity and accelerometer-bias prior (tslam_ba_inertial) before
        the batch is submitted.  One stereo pair: in pair 0's rectified-left camera; a rig: in the
        body (base_link) frame of its body window (pair = n_pairs), the filter's camera-0 vectors
        rotated into it (the velocity only seeds the solve)."""
        cfg, imu = self._config, self._imu
        if not self._ine_on():
            return
        rig = len(self._pairs) > 1
        pair = len(self._pairs) if rig else 0
        R0 = self._base_T_rects[0][:3, :3]   # base_R_rect0: camera-0 vectors into the body world
        st = imu.st
        g = imu.gravity()
        self._handle.ba_inertial(R0 @ g if rig else g, st.ba, 1.0 / max(st.var_b, 1e-12), st.bg,
                                 1.0 / max(st.var_g, 1e-12), pair=pair)
        floors = dict(r_floor=cfg.ba_inertial_r_floor, ba_floor=cfg.ba_inertial_ba_floor, bg_floor=cfg.ba_inertial_bg_floor)
        g = self._handle.frames_done
        for k, (step, smp) in enumerate(zip(steps, samples)):
            gk = g + k
            if step is None or step.v1 is None or smp[0] is None:
                self._kf_ine = None
            else:
                if self._kf_ine is None:
                    self._kf_ine = ([], gk, None)
                self._kf_ine[0].append(smp)
            if gk % cfg.ba_kf_interval == 0:
                acc = self._kf_ine
                if acc is not None and acc[1] == gk - cfg.ba_kf_interval + 1 and len(acc[0]) == cfg.ba_kf_interval:
                    if rig:
                        rec = imu.preintegrate(acc[0], st.bg, st.ba, None if acc[2] is None else R0 @ acc[2],
                                               cfg.ba_inertial_v_floor, cfg.ba_inertial_p_floor,
                                               frame_R_imu=self._base_T_imu[:3, :3], lever=self._base_T_imu[:3, 3],
                                               **floors)
                        self._handle.ba_inertial_factor(gk, rec, R0 @ step.v1, pair=pair)
                    else:
                        rec = imu.preintegrate(acc[0], st.bg, st.ba, acc[2], cfg.ba_inertial_v_floor,
                                               cfg.ba_inertial_p_floor, **floors)
                        self._handle.ba_inertial_factor(gk, rec, step.v1)
                self._kf_ine = ([], gk + 1, None if step is None else step.w.copy())

    def _set_motion_prior(self, *args) -> None:
        """The batch's priors on the handle (every rank's handle on a sharded rig: each refines its
        frame range and chains the whole batch)."""
        for h in (self._shard["handles"] if self._shard is not None else [self._handle]):
            h.set_motion_prior(*args)

    def process_batch(self, images, timestamps: list[float] | None = None, stream=None) -> dict:
        """Throughput entry: ``images`` is a device uint8 tensor already in HBM: [n, 2P, H, W] gray
        stereo pairs, or [n, P, 5*H*W] RGB-D records (``rgbd.pack_rgbd``)."""
        if self._handle is None:
            raise RuntimeError("Not initialized")
        if self._shard is not None:
            raise RuntimeError("process_batch takes one device's images; a sharded rig (devices) uses process_frames")
        n = int(images.shape[0])
        s = stream if stream is not None else self._torch.cuda.current_stream(self._device)
        self.flush()
        self._handle.submit(images.data_ptr(), n, s.cuda_stream)
        self._integrate_depth(images.data_ptr(), n, s.cuda_stream)
        res = self._read(n)
        self._publish(res, timestamps or [float(i) for i in range(n)], self._handle.frames_done - n)
        return res

    # -- RGB-D dense mapping ----------------------------------------------
    def _integrate_depth(self, records_ptr: int, n: int, stream: int, cams_per_frame: int | None = None) -> None:
        """The batch's depth images of pair 0 into the TSDF volume, with the batch's device-resident
        tracked poses (untracked frames are skipped), on the batch's stream.  ``cams_per_frame``: the
        records per frame of the buffer (a sharded rig: rank 0's cameras, pair 0 first)."""
        if not self._config.dense_map:
            return
        r = self._rects[0]
        hw = r.width * r.height
        stride = 5 * hw * (cams_per_frame or len(self._pairs))
        if self._config.dense_color:   # the record's BGR part with its depth part
            self._handle.tsdf_integrate_rgbd(records_ptr, records_ptr + 3 * hw, stride, n,
                                             first_frame=self._handle.frames_done - n, pair=0, stream=stream)
        else:
            self._handle.tsdf_integrate(records_ptr + 3 * hw, stride, n,
                                        first_frame=self._handle.frames_done - n, pair=0, stream=stream)

    def get_dense_map(self) -> dict | None:
        """The TSDF volume (nvblox-shaped): ``tsdf`` / ``weight`` f32 [nz][ny][nx] (metres of
        truncated signed distance; weight 0 = never observed), the voxel grid (``origin``,
        ``voxel_size``, voxel (i, j, k) centred at origin + voxel_size (i, j, k) + voxel_size / 2 in
        the tracking world) and ``world_T_volume`` (4x4: that frame in the published world =
        base_link at the first frame).  None unless ``dense_map`` is on.  Synchronises."""
        cfg = self._config
        if not cfg.dense_map or self._handle is None:
            return None
        self.flush()
        tsdf, weight = self._handle.tsdf_read()
        out = {}
        if cfg.dense_color:
            out["color"], out["color_weight"] = self._handle.tsdf_read_color()
        return {**out, "tsdf": tsdf, "weight": weight, "origin": np.array(cfg.tsdf_origin, dtype=np.float64),
                "voxel_size": float(cfg.voxel_size),
                "truncation_m": cfg.tsdf_integrator_truncation_distance_vox * cfg.voxel_size,
                "world_T_volume": self._map_offset @ self._base_T_rect}

    def get_mesh(self) -> dict | None:
        """The surface mesh of the TSDF volume (marching cubes on the device, k_dense.hip):
        ``triangles`` f32 [n][3][3] (metres in the tracking world, facing free space), with the
        colour layer ``colors`` f32 [n][3][3] (R, G, B per vertex), and ``world_T_volume``.  None unless ``dense_map`` is on.  Synchronises."""
        cfg = self._config
        if not cfg.dense_map or self._handle is None:
            return None
        self.flush()
        if cfg.dense_color:
            tris, cols = self._handle.mesh(cfg.mesh_integrator_min_weight, colors=True)
            return {"triangles": tris, "colors": cols, "world_T_volume": self._map_offset @ self._base_T_rect}
        return {"triangles": self._handle.mesh(cfg.mesh_integrator_min_weight),
                "world_T_volume": self._map_offset @ self._base_T_rect}

    def get_esdf(self) -> dict | None:
        """The Euclidean signed distance field of the volume (k_dense.hip): ``esdf`` f32
        [nz][ny][nx] (metres, negative inside, +-esdf_integrator_max_distance_m beyond it, NaN
        unobserved) on the TSDF grid.  None unless ``dense_map`` is on.  Synchronises."""
        cfg = self._config
        if not cfg.dense_map or self._handle is None:
            return None
        self.flush()
        esdf = self._handle.esdf(cfg.esdf_integrator_max_distance_m, cfg.esdf_integrator_max_site_distance_vox,
                                 cfg.esdf_integrator_min_weight)
        return {"esdf": esdf, "origin": np.array(cfg.tsdf_origin, dtype=np.float64), "voxel_size": float(cfg.voxel_size),
                "world_T_volume": self._map_offset @ self._base_T_rect}

    def get_esdf_slice(self) -> dict | None:
        """nvblox's 2-D distance map: unsigned distance f32 [nz][nx] to the nearest surface voxel of
        the height band [esdf_slice_min_height, esdf_slice_max_height) (tracking-world y), NaN
        where the band was never observed.  None unless ``dense_map`` is on.  Synchronises."""
        cfg = self._config
        if not cfg.dense_map or self._handle is None:
            return None
        self.flush()
        s, y_org, ny = cfg.voxel_size, cfg.tsdf_origin[1], int(cfg.tsdf_dims[1])
        y0 = int(np.clip(np.floor((cfg.esdf_slice_min_height - y_org) / s), 0, ny - 1))
        y1 = int(np.clip(np.ceil((cfg.esdf_slice_max_height - y_org) / s), y0 + 1, ny))
        dist = self._handle.esdf_slice(y0, y1, cfg.esdf_integrator_max_distance_m,
                                       cfg.esdf_integrator_max_site_distance_vox, cfg.esdf_integrator_min_weight)
        return {"distance": dist, "band": (y0, y1), "origin": np.array(cfg.tsdf_origin, dtype=np.float64),
                "voxel_size": float(s), "world_T_volume": self._map_offset @ self._base_T_rect}

    def _read(self, n: int) -> dict:
        res = self._handle.read_poses(n)
        if len(self._pairs) > 1:
            res["rig"] = self._handle.read_rig_poses(n)
        return res

    def _body_pose(self, res: dict, k: int) -> tuple[int, np.ndarray, np.ndarray]:
        """(status, world_T_base, 6x6 body covariance) of frame k of a batch result."""
        bt = self._base_T_rect
        stats = res["stats"][k, :, 0]
        if len(self._pairs) == 1:
            status = int(stats[0])
            body = bt @ res["T_abs"][k, 0] @ self._bt_inv
            ad = self._bt_ad   # camera-frame twist -> base-frame twist (rotation and lever arm)
            cov = ad @ res["cov"][k, 0] @ ad.T if status == POSE_OK else np.zeros((6, 6))
            return status, body, cov
        # multi-pair rig: the device's generalised PnP over all pairs (k_rig_pose), already in the
        # base frame and chained (world = base_link at the first frame)
        rig = res["rig"]
        status = int(rig["stats"][k, 0])
        cov = rig["cov"][k] if status == POSE_OK else np.zeros((6, 6))
        return status, rig["T_abs"][k].copy(), cov

    def _ba_corrections(self, res: dict, n: int, g0: int):
        """Per frame of the batch: the correction W_ba(kf) inv(W_fe(kf)) (or None) — rect-left
        world_T_cam terms for one pair, world_T_body (base) terms for a rig's body window."""
        cfg = self._config
        if cfg.ba_window <= 0:
            return None
        P = len(self._pairs)
        rig = P > 1
        for k in range(n):
            if (g0 + k) % cfg.ba_kf_interval == 0:
                self._fe_at[g0 + k] = (res["rig"]["T_abs"][k] if rig else res["T_abs"][k, 0]).copy()
        win = self._handle.ba_read(P if rig else 0)
        self._ba_window = win
        self._ba_pairs = [self._handle.ba_read(q) for q in range(P)] if rig else [win]
        for q, w in enumerate(self._ba_pairs):
            self._accumulate_map(w, q)
        live = {}
        for s_, f in enumerate(win["frames"]):
            if f >= 0:
                live[int(f)] = _invert(win["T_cw"][s_])
                self._kf_final[int(f)] = live[int(f)]
        for f in [f for f in self._fe_at if f not in live and f < min(live, default=0)]:
            del self._fe_at[f]   # evicted: its final estimate is kept in _kf_final
        if not live:
            return None
        frames = sorted(live)
        out = []
        for k in range(n):
            g = g0 + k
            kf = max([f for f in frames if f <= g], default=frames[0])
            out.append(live[kf] @ _invert(self._fe_at[kf]))
        return out

    def _accumulate_map(self, win: dict, pair: int = 0) -> None:
        """Merge a window's landmarks (latest BA positions) into the persistent map by global id
        (rect-left frame of pair 0; a rig's pairs keep theirs apart: key gid * n_pairs + pair).
        ``SlamConfig.enable_mapping`` off keeps no map; ``max_map_size`` bounds it (the landmarks
        updated longest ago go first; interface.py:110-111)."""
        cfg = self._config
        if not cfg.enable_mapping:
            return
        mp = self._handle.ba_read_map(pair)
        P = len(self._pairs)
        to_rect0 = _invert(self._base_T_rect) if P > 1 else np.eye(4)   # a rig's BA world is the base frame
        occ = win["frames"] >= 0
        ids, counts = np.unique(win["lm"][occ], return_counts=True)
        keep = ids >= 0
        for i, n in zip(ids[keep], counts[keep]):
            x = to_rect0[:3, :3] @ win["X"][i] + to_rect0[:3, 3]
            key = int(mp["gid"][i]) * P + pair
            self._map_points.pop(key, None)   # re-inserted: most recently updated last
            self._map_points[key] = (x, mp["desc"][i].copy(), int(n))
        while len(self._map_points) > max(int(cfg.max_map_size), 0):
            del self._map_points[next(iter(self._map_points))]

    def _publish(self, res: dict, stamps: list[float], g0: int) -> None:
        with self._map_lock:
            self._publish_locked(res, stamps, g0)

    def _publish_locked(self, res: dict, stamps: list[float], g0: int) -> None:
        entry = next((e for e in self._imu_batches if e["res"] is None), None) if self._imu is not None else None
        if entry is not None and "samples" not in entry:
            entry["res"] = ()
        elif entry is not None:   # what the filter absorbs of the tracked motions (at the next prior that may use it)
            steps = entry["steps"]
            if len(self._pairs) == 1:   # the vision-only motion behind each prior-weighted solution
                st = res["stats"][:, 0]
                sig = np.ascontiguousarray(st[:, 6:8]).view(np.float64)[:, 0]   # sigma^2 (tslam.h)
                t_rel, cov = res["T_rel"][:, 0].copy(), res["cov"][:, 0].copy()
                for k, step in enumerate(steps[:len(st)]):
                    if step is not None and int(st[k, 0]) == POSE_OK:
                        t_rel[k], cov[k] = vision_only(t_rel[k], cov[k], float(sig[k]), step)
                entry["res"] = (st[:, 0].copy(), t_rel, cov)
            else:   # the rig's body motion, moved into pair 0's camera (the filter's frame)
                e0 = self._base_T_rects[0]
                ie0, ad = _invert(e0), adjoint(_invert(e0))
                rig = res["rig"]
                t_rel = np.stack([ie0 @ m @ e0 for m in rig["T_rel"]])
                cov = np.stack([ad @ c @ ad.T for c in rig["cov"]])
                entry["res"] = (rig["stats"][:, 0].copy(), t_rel, cov)
        latest = None
        state = self._state
        corr = self._ba_corrections(res, len(stamps), g0)
        bt, bt_inv = self._base_T_rect, self._bt_inv
        for k, ts in enumerate(stamps):
            status, body, cov = self._body_pose(res, k)
            if corr is not None and status != POSE_LOST:   # a rig's correction is in body terms
                body = corr[k] @ body if len(self._pairs) > 1 else bt @ corr[k] @ res["T_abs"][k, 0] @ bt_inv
            if isinstance(self._loop, _AsyncLoop):   # oracle/numpy_loop.py LoopPolicy.step
                g = g0 + k
                raw = bt_inv @ body @ bt                           # rect-left world_T_cam before loop correction
                self._loop.observe(g, status)
                if status == POSE_OK and g % self._config.loop_kf_interval == 0:
                    self._loop.node(g, raw, ts)
                self._loop.advance(until=g)
                body = bt @ self._loop.corr @ raw @ bt_inv
                if self._loop.reloc:   # no pose until the new segment is anchored in the map
                    state = TrackingState.RELOCALIZING
                    latest = None
                    continue
            elif self._loop is not None and status != POSE_LOST:
                g = g0 + k
                raw = bt_inv @ body @ bt                           # rect-left world_T_cam before loop correction
                if status == POSE_OK and g % self._config.loop_kf_interval == 0:
                    self._loop_keyframe(g, raw, ts)
                body = bt @ self._loop.corr @ raw @ bt_inv
            body = self._map_offset @ body
            if status == POSE_LOST:
                state = TrackingState.LOST
                latest = None
                continue
            state = TrackingState.TRACKING if status == POSE_OK else TrackingState.INITIALIZING
            latest = SlamPose(
                position=body[:3, 3].copy(),
                rotation=_quat_xyzw(body),
                timestamp=ts,
                tracking_state=state,
                confidence=confidence_from_covariance(cov) if status == POSE_OK else 1.0,
                covariance=cov,
            )
            if status == POSE_INIT:
                self._keyframe_poses.append(latest)
            g = g0 + k
            if self._config.ba_window > 0 and g % self._config.ba_kf_interval == 0:
                self._kf_stamp[g] = ts
        with self._pose_lock:
            self._latest_pose = latest
            self._state = state
        self._last_result = res

    # -- loop closure + keyframe pose graph ---------------------------
    def _loop_keyframe(self, g: int, raw: np.ndarray, ts: float) -> None:
        """Keyframe g: store every pair's view of it in the device database (entry idx * P + p),
        add its odometry edge, look for a loop among the keyframes at least ``loop_min_gap`` older
        (signature votes of each pair's entry against every older entry of every pair; the best
        vote wins, lower pair first), verify it (RANSAC on the voting pair's camera against the
        entry's landmarks) and, on a verified loop, re-solve the pose graph on the device.  A
        pair-q view of a place pair p saw gives the node edge in pair 0's frame:
        T_c^-1 T_q = M_p V^-1 M_q^-1 with V = cam_q_T_cam_p and M_p = rect0_T_rect_p."""
        cfg, lp, h = self._config, self._loop, self._handle
        idx, P = len(lp.frames), len(self._pairs)
        if idx >= cfg.loop_max_keyframes:
            if not lp.full:
                logger.warning("loop closure: keyframe database full (%d); no further keyframes", idx)
                lp.full = True
            return
        slots = [h.loop_add_keyframe(g, pair=p)[0] for p in range(P)]
        assert slots == list(range(idx * P, idx * P + P))
        info = lp.information(cfg)
        if idx == 0:
            T = lp.corr @ raw
        else:
            Z = _invert(lp.raw[-1]) @ raw
            T = lp.T[-1] @ Z
            lp.edges.append((idx - 1, idx))
            lp.meas.append(Z)
            lp.info.append(info)
        lp.frames.append(g)
        lp.stamps.append(ts)
        lp.raw.append(raw.copy())
        lp.T.append(T)
        n_allowed = idx - cfg.loop_min_gap + 1
        if n_allowed <= 0:
            return
        best, q, e = -1, 0, 0
        for p, slot in enumerate(slots):
            votes = h.loop_query(slot, n_allowed * P)
            j = int(np.argmax(votes))
            if votes[j] > best:
                best, q, e = int(votes[j]), p, j
        if best < cfg.loop_min_votes:
            return
        ver = h.loop_verify(g, e, pair=q)
        if int(ver["stats"][0]) != POSE_OK or int(ver["stats"][2]) < cfg.loop_min_inliers:
            return
        j, p = divmod(e, P)
        m = [_invert(self._base_T_rects[0]) @ self._base_T_rects[k] for k in (p, q)]
        meas = m[0] @ _invert(ver["T"]) @ _invert(m[1])
        try:
            sol = h.pose_graph(np.stack(lp.T), np.array(lp.edges + [(j, idx)]), np.stack(lp.meas + [meas]),
                               np.stack(lp.info + [info]), cfg.pg_iters)
        except SingularSystemError as exc:   # LoopPolicy's rejection: the loop is dropped, tracking goes on
            logger.warning("loop closure: keyframe %d -> %d rejected (%s)", lp.frames[j], g, exc)
            return
        lp.edges.append((j, idx))
        lp.meas.append(meas)
        lp.info.append(info)
        lp.loops.append((lp.frames[j], g, int(ver["stats"][2])))
        lp.pairs.append((p, q))
        lp.T = list(sol["T"])
        lp.cost = sol["cost"]
        lp.corr = lp.T[-1] @ _invert(raw)
        logger.info("loop closure: keyframe %d -> %d (%d inliers), pose graph cost %.3g", lp.frames[j], g,
                    int(ver["stats"][2]), sol["cost"])

    @property
    def loop_closures(self) -> list[tuple[int, int, int]]:
        """Verified loops so far: (older keyframe frame, newer keyframe frame, inliers)."""
        return list(self._loop.loops) if self._loop is not None else []

    @property
    def pose_graph(self) -> dict | None:
        """The keyframe pose graph: frames, world_T_cam (rect-left) per node, edges (a, b)."""
        if self._loop is None:
            return None
        lp = self._loop
        return {"frames": list(lp.frames), "T": np.array(lp.T).reshape(-1, 4, 4), "edges": list(lp.edges),
                "meas": [m.copy() for m in lp.meas], "cost": lp.cost}

    # ------------------------------------------------------------------------------------------
    def get_tracking_state(self) -> TrackingState:
        return self._state

    def get_map(self) -> SlamMap:
        """Without BA: the (re)initialisation poses.  With BA: every keyframe so far at its latest
        BA estimate (world_T_base) and the landmarks of every pair's window (world frame, with their
        observation counts).  Safe to call from another thread while process_frames runs."""
        with self._map_lock:
            return self._get_map_locked()

    def _get_map_locked(self) -> SlamMap:
        if self._loop is not None and self._loop.frames and (self._config.ba_window <= 0 or self._ba_window is None):
            bt = self._base_T_rect
            kfs = []
            for T, ts in zip(self._loop.T, self._loop.stamps):
                body = self._map_offset @ bt @ T @ _invert(bt)
                kfs.append(SlamPose(position=body[:3, 3].copy(), rotation=Rotation.from_matrix(body[:3, :3]).as_quat(),
                                    timestamp=ts, tracking_state=TrackingState.TRACKING, confidence=1.0))
            smap = SlamMap(keyframe_poses=kfs)
        elif self._config.ba_window <= 0 or self._ba_window is None:
            smap = SlamMap(keyframe_poses=list(self._keyframe_poses))
        else:
            rig = len(self._pairs) > 1   # body window: keyframes are already world_T_base, landmarks in base
            bt = np.eye(4) if rig else self._base_T_rect
            kfs = []
            for f in sorted(self._kf_final):
                body = bt @ self._kf_final[f] @ _invert(bt)
                kfs.append(SlamPose(position=body[:3, 3].copy(), rotation=Rotation.from_matrix(body[:3, :3]).as_quat(),
                                    timestamp=self._kf_stamp.get(f, float(f)), tracking_state=TrackingState.TRACKING,
                                    confidence=1.0))
            points = []
            for win in self._ba_pairs:
                occ = win["frames"] >= 0
                ids, counts = np.unique(win["lm"][occ], return_counts=True)
                keep = ids >= 0
                ids, counts = ids[keep], counts[keep]
                pts = win["X"][ids] @ bt[:3, :3].T + bt[:3, 3]
                points += [MapPoint(position=p.copy(), observations=int(c)) for p, c in zip(pts, counts)]
            # SlamConfig.enable_mapping / max_map_size (interface.py:110-111)
            points = points[:max(int(self._config.max_map_size), 0)] if self._config.enable_mapping else []
            smap = SlamMap(points=points, keyframe_poses=kfs)
        pose = self._latest_pose
        if pose is not None:
            smap.timestamp = pose.timestamp
        return smap

    # -- map persistence / relocalisation (interface.py:228-256) -----------
    def save_map(self, path: str) -> bool:
        """Write the landmarks gathered by local BA (world = base_link frame, rBRIEF descriptors,
        global ids, observation counts) and every keyframe pose to ``path`` (NumPy .npz, no
        pickles).  False when there is nothing to save (local BA off or no landmark yet)."""
        with self._map_lock:
            return self._save_map_locked(path)

    def _save_map_locked(self, path: str) -> bool:
        if not self._map_points or self._handle is None:
            return False
        bt = self._base_T_rect
        gids = np.array(sorted(self._map_points), dtype=np.int64)
        xyz = np.stack([self._map_points[g][0] for g in gids])
        desc = np.stack([self._map_points[g][1] for g in gids]).astype(np.uint32)
        obs = np.array([self._map_points[g][2] for g in gids], dtype=np.int64)
        smap = self.get_map()
        kf = np.stack([p.to_4x4_matrix() for p in smap.keyframe_poses]) if smap.keyframe_poses else np.zeros((0, 4, 4))
        with open(path, "wb") as fh:
            np.savez(fh, points=xyz @ bt[:3, :3].T + bt[:3, 3], desc=desc, gid=gids, observations=obs,
                     keyframe_world_T_base=kf, keyframe_stamps=np.array([p.timestamp for p in smap.keyframe_poses]),
                     base_T_rect=bt)
        return True

    def load_map(self, path: str) -> bool:
        """Load a map written by ``save_map`` and upload it for ``relocalize``."""
        if self._handle is None:
            raise RuntimeError("Not initialized")
        try:
            with np.load(path, allow_pickle=False) as z:
                pts, desc = np.asarray(z["points"], dtype=np.float64), np.asarray(z["desc"], dtype=np.uint32)
        except (OSError, KeyError, ValueError) as exc:
            logger.warning("load_map(%s) failed: %s", path, exc)
            return False
        if len(self._pairs) > 1:   # a rig relocalises in the base frame from every pair (tslam_relocalize_rig)
            self._handle.map_upload(pts, desc)
        else:
            inv_bt = _invert(self._base_T_rect)
            self._handle.map_upload(pts @ inv_bt[:3, :3].T + inv_bt[:3, 3], desc)   # into the rect-left frame
        self._map_loaded = True
        return True

    def relocalize(self) -> bool:
        """Pose the latest processed frame in the loaded map (descriptor matching + P3P-RANSAC on
        the device; a rig: every pair's view, joined by the rig pose, so a map any one pair saw
        relocalises it); on success the published poses continue in the map's world frame."""
        if self._handle is None:
            raise RuntimeError("Not initialized")
        if not self._map_loaded or self._handle.frames_done == 0:
            return False
        self.flush()
        if len(self._pairs) > 1:   # every pair matches the map; the rig pose solves the body
            res = self._handle.relocalize_rig(self._handle.frames_done - 1)
            if int(res["stats"][0]) != POSE_OK:
                return False
            map_pose = _invert(res["T"])                                 # map world_T_base of that frame
        else:
            res = self._handle.relocalize(self._handle.frames_done - 1)
            if int(res["stats"][0]) != POSE_OK:
                return False
            bt = self._base_T_rect
            map_pose = bt @ _invert(res["T"]) @ _invert(bt)              # map world_T_base of that frame
        with self._pose_lock:
            cur = self._latest_pose
        session = (_invert(self._map_offset) @ cur.to_4x4_matrix()) if cur is not None else np.eye(4)
        self._map_offset = map_pose @ _invert(session)
        if cur is not None:
            body = map_pose
            with self._pose_lock:
                self._latest_pose = SlamPose(position=body[:3, 3].copy(), rotation=Rotation.from_matrix(body[:3, :3]).as_quat(),
                                             timestamp=cur.timestamp, tracking_state=TrackingState.TRACKING,
                                             confidence=cur.confidence, covariance=cur.covariance)
                self._state = TrackingState.TRACKING
        return True

    def reset(self) -> None:
        self._in_flight = 0
        with self._pose_lock:
            self._latest_pose = None
        self._staged, self._staged_imu, self._prev_stamp = [], [], None
        self._imu_batches = []
        self._imu_seq = 0
        self._kf_imu = None
        self._kf_ine = None
        if self._imu is not None:
            self._imu.reset()
        self._keyframe_poses = []
        self._fe_at, self._kf_final, self._kf_stamp, self._ba_window, self._ba_pairs = {}, {}, {}, None, []
        self._map_points, self._map_offset = {}, np.eye(4)
        if isinstance(self._loop, _AsyncLoop):
            self._loop = _AsyncLoop(self._handle, self._config, self._loop.P, self._loop.m)
        elif self._loop is not None:
            self._loop = _LoopGraph()
        if self._shard is not None:
            self._shard["stamps"].clear()
        for h in (self._shard["handles"] if self._shard is not None else [self._handle] if self._handle else []):
            h.reset()
        self._state = TrackingState.INITIALIZING
        self._frame_count = 0

    def shutdown(self) -> None:
        if self._handle is not None and (self._staged or self._in_flight):
            try:   # the tail of the stream: staged frames run as a short last batch and are published
                self.flush()
            except RuntimeError as exc:
                logger.warning("shutdown: the last %d staged frame(s) were not tracked: %s", len(self._staged), exc)
        if self._shard is not None:
            self._shard["group"].close()
            for h in self._shard["handles"]:
                h.close()
            self._shard = None
            self._handle = None
        if self._handle is not None:
            self._handle.close()
            self._handle = None
        self._state = TrackingState.NOT_INITIALIZED

    @property
    def frame_count(self) -> int:
        return self._frame_count

    @property
    def num_cameras(self) -> int:
        return self._num_cameras

    @property
    def handle(self) -> Handle | None:
        return self._handle

    @property
    def rectifications(self) -> list[StereoRectification]:
        return list(self._rects)
