"""Throughput bench: synced stereo frames/sec (detect + match + pose) @ 640x400 on MI355X.

python bench.py --gpus N --steps K --warmup W   (N > 1 under torch.distributed.run, one rank/GPU)
python bench.py --config c3 [--gpus N]          (BASELINE.json configs[2]: 4-OAK bracket rig, 8 streams)
python bench.py --config c4                     (BASELINE.json configs[3]: 1280x800, K=4000, + local BA)
python bench.py --config c5 [--gpus 4]          (BASELINE.json configs[4]: 4-camera RGB-D rig 1280x720, one camera per GPU)

* N = 1, config c2 (BASELINE.json configs[1]): one stereo pair 640x400, K=2000 ORB-style
  keypoints per image, synthetic room sequence; a *step* = one batch of ``--batch`` synchronised
  stereo frames pushed through the whole hot path (rectify -> pyramid -> FAST/NMS/top-K ->
  orientation + rBRIEF -> stereo + temporal Hamming match -> sub-pixel refinement -> P3P-RANSAC
  -> Gauss-Newton -> pose chaining).
* N > 1 (c2): one camera STREAM per GPU (BASELINE.json north_star): N streams =
  N/2 stereo sources of the bracket rig (scripts/run_slam.py:45-50, brackets.urdf joints), the
  sharded rig of thor_slam_amd/shard.py (front end per stream, RCCL all-to-all of raw images +
  stream blocks, per-pair back end + rig pose on each rank's frame range, all-gather of pose
  records).  value = synced stereo (pair) frames/s of the whole rig; weak scaling (one stream
  per GPU).
* c3: the 4-source bracket rig (8 streams, 4 pairs) sharded over --gpus N (N = 1: one handle);
  value = rig frames/s (one frame = all 8 images); strong scaling.
* inputs are rendered on the host before timing and are resident in HBM (a triangle-wave
  replay of ``--unique`` rendered frames, so consecutive frames stay consecutive in time).
* timing: barrier + synchronize on both sides of exactly K steps; MAX over ranks.
* roofline: per-kernel HIP-event timing of the timed steps on the stream each kernel runs on,
  for the dominant kernel: algorithmic bytes / average duration vs 8 TB/s.
* cpu_baseline (rank 0, N = 1): the NumPy oracle on a bounded sample of the same frames, over
  the host cores this process may use, plus the one-process figure.
* boundary (c2, N = 1): HipSlamEngine.process_frames on host SynchronizedFrameSets from the
  CameraRig (the drop-in boundary, scripts/run_slam.py:314-328) at batch 1 and 64.
* --config c4: the same step plus the A8 stage (every 5th frame a keyframe of a 10-keyframe
  window, 5 Gauss-Newton iterations per keyframe); the roofline is then that of the dominant
  kernel of the step, the FP64-MFMA Schur product when it dominates (HIP events around its launches).
* --config c5: the 4-camera RGB-D rig (BGR u8 + aligned u16 mm depth, 1280x720 per camera, the
  cameras on the brackets.urdf joints): per camera the colour image is converted on the device,
  depth replaces stereo matching, and every frame gets the rig pose over all 4 cameras.  N = 1:
  one handle for the whole rig; N = 2 / 4: the cameras sharded over the GPUs (each rank tracks its
  own cameras, RCCL all-to-all of pair blocks, rig pose per frame range, pose all-gather); value =
  rig frames/s, strong scaling.
"""

from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time
from concurrent.futures import ProcessPoolExecutor
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
for _p in (ROOT, ROOT / "thor-slam_amd"):
    if str(_p) not in sys.path:
        sys.path.insert(0, str(_p))

METRIC = "synced stereo frames/sec (detect+match+pose) @640×400, 1/2/4/8 GPU"
METRIC_C3 = "synced rig frames/sec (4 stereo pairs = 8 streams, detect+match+pose+rig pose) @640×400, 1/2/4/8 GPU"
METRIC_C4 = "synced stereo frames/sec (detect+match+pose+10-keyframe local BA) @1280×800, 1 GPU"
METRIC_C5 = "RGB-D rig frames/sec (4 cameras, BGR+depth, detect+match+pose+rig pose) @1280×720, 1/2/4 GPU"
HBM_PEAK_GBS = 8000.0
# VALU issue: 256 CUs x 4 SIMD-32, a wave64 instruction every 2 cycles per SIMD at 2.4 GHz
VALU_PEAK_WINST = 256 * 4 * 2.4e9 / 2
# C2 frames per step: larger batches amortise each launch's ramp and drain (measured on one MI355X,
# round 2: 147.3k / 153.3k / 154.0k / 155.3k frames/s at B = 256 / 512 / 768 / 1024; round 5, two
# runs each: 239.1k / 242.1k / 243.9k at B = 1024 / 2048 / 4096 — 2048 takes most of the gain at
# half the step latency of 4096)
C2_BATCH = 2048
# C2 distinct rendered frames (triangle-wave replay): the input working set exceeds the MALL
C2_UNIQUE = 1024
# C5 rig frames per step: 4 periods of the 24-frame triangle wave (the resident batch is replayed)
C5_BATCH = 184
# C3 rig frames per step (one GPU, and each step of the sharded rig): 1024, as C2 — at 8 ranks a
# rank's back end then solves 128 frames, not 32 (the per-frame latency chains of the pose and rig
# kernels stop dominating; tools/shard_probe.py: 1-GPU step / per-GPU step 6.1-6.7 at 1024 against
# 4.2-4.5 at 256, profiles/r4e_probe_c3_w8_b*.json)
C3_BATCH = 1024
FP64_MFMA_PEAK_TFS = 78.6   # MI355X FP64 matrix peak (AMD spec; the microarch guide lists no FP64 row)
# bench kernel label -> device symbol (rocprofv3 / PMC summaries); "pose" is k_corr+k_ransac+k_refine
KERNEL_SYMBOL = {"rectify_pyramid": "k_rectify_pyramid", "detect": "k_detect", "select": "k_select",
                 "describe": "k_describe", "match": "k_match", "match_refine": "k_refine_temporal",
                 "pose": "k_ransac", "chain": "k_chain", "rig": "k_rig_pose"}
# the bracket rig of scripts/run_slam.py:45-50 (CAMERA_MAP), global camera order = sorted names
RIG_SOURCES = ("192.168.2.21", "192.168.2.22", "192.168.2.23", "192.168.2.25")
JOINTS = ROOT / "tests" / "golden" / "brackets_joints.json"   # brackets.urdf joints (tests/test_boundary.py pins them)


# ---- rendering ------------------------------------------------------------------------------
def _render_chunk(args):
    seed, idx, width, height = args
    from thor_slam_amd.synthetic import SyntheticStereoSource

    src = SyntheticStereoSource(seed=seed, n_frames=max(idx) + 1, width=width, height=height)
    return [src.render_stereo_sequence(1, start=i)[0] for i in idx]


def render_frames(seed: int, n: int, workers: int, width: int = 640, height: int = 400) -> np.ndarray:
    idx = list(range(n))
    chunks = [idx[i::workers] for i in range(workers) if idx[i::workers]]
    out = np.empty((n, 2, height, width), dtype=np.uint8)
    if workers <= 1:
        for c in chunks:
            for i, fr in zip(c, _render_chunk((seed, c, width, height))):
                out[i] = fr
        return out
    with ProcessPoolExecutor(max_workers=workers) as ex:
        for c, frs in zip(chunks, ex.map(_render_chunk, [(seed, c, width, height) for c in chunks])):
            for i, fr in zip(c, frs):
                out[i] = fr
    return out


def rig_setup(names, width: int = 640, height: int = 400):
    """Bracket rig of `names`: sources, flat camera list, stereo pairs, rectifications, base_T_rect-left."""
    from thor_slam_amd.calib import extract_cameras, stereo_pairs, stereo_rectify
    from thor_slam_amd.synthetic import synthetic_rig

    joints = json.loads(JOINTS.read_text())
    srcs, rig = synthetic_rig(joints, names, width, height)
    cams = extract_cameras(rig.calibration, 2 * len(names))
    pairs = stereo_pairs(cams)
    rects = [stereo_rectify(cams[l], cams[r]) for l, r in pairs]
    E = [cams[l].extrinsics.to_4x4_matrix() @ r.left_optical_T_rect() for (l, _), r in zip(pairs, rects)]
    return srcs, cams, pairs, rects, E


def _render_rig_chunk(args):
    names, items, width, height = args   # items: (frame, global camera)
    srcs, cams, _, _, _ = rig_setup(names, width, height)
    by = {s.name: s for s in srcs}
    return [by[cams[c].source_name].render_image(i, cams[c].cam_idx) for i, c in items]


def render_rig_frames(names, n: int, cam_lo: int, cam_hi: int, workers: int, width: int = 640,
                      height: int = 400) -> np.ndarray:
    """[n][cam_hi - cam_lo][H][W] u8 of the rig's global cameras cam_lo .. cam_hi-1."""
    items = [(i, c) for i in range(n) for c in range(cam_lo, cam_hi)]
    chunks = [items[k::workers] for k in range(workers) if items[k::workers]]
    out = np.empty((n, cam_hi - cam_lo, height, width), dtype=np.uint8)
    with ProcessPoolExecutor(max_workers=max(1, len(chunks))) as ex:
        for ch, imgs in zip(chunks, ex.map(_render_rig_chunk, [(tuple(names), ch, width, height) for ch in chunks])):
            for (i, c), img in zip(ch, imgs):
                out[i, c - cam_lo] = img
    return out


def rgbd_rig_setup(names, width: int = 1280, height: int = 720):
    """RGB-D rig of `names` on the bracket joints: sources, flat camera list, (colour, depth)
    pairs, undistortions, base_T_cam of each colour camera."""
    from thor_slam_amd.calib import extract_cameras, rgbd_pairs, rgbd_undistort
    from thor_slam_amd.synthetic import synthetic_rgbd_rig

    joints = json.loads(JOINTS.read_text())
    srcs, rig = synthetic_rgbd_rig(joints, names, width, height)
    cams = extract_cameras(rig.calibration, 2 * len(names))
    pairs = rgbd_pairs(cams)
    rects = [rgbd_undistort(cams[c]) for c, _ in pairs]
    E = [cams[c].extrinsics.to_4x4_matrix() @ r.left_optical_T_rect() for (c, _), r in zip(pairs, rects)]
    return srcs, cams, pairs, rects, E


def _render_rgbd_chunk(args):
    names, items, width, height = args   # items: (frame, rig camera = pair index)
    from thor_slam_amd.rgbd import pack_rgbd

    srcs, cams, pairs, _, _ = rgbd_rig_setup(names, width, height)
    by = {s.name: s for s in srcs}
    return [pack_rgbd(*by[cams[pairs[q][0]].source_name].render_rgbd(i)) for i, q in items]


def render_rgbd_rig_frames(names, n: int, cam_lo: int, cam_hi: int, workers: int, width: int = 1280,
                           height: int = 720) -> np.ndarray:
    """[n][cam_hi - cam_lo][5*H*W] u8 device records of the RGB-D rig's cameras cam_lo .. cam_hi-1."""
    items = [(i, c) for i in range(n) for c in range(cam_lo, cam_hi)]
    chunks = [items[k::workers] for k in range(workers) if items[k::workers]]
    out = np.empty((n, cam_hi - cam_lo, 5 * width * height), dtype=np.uint8)
    with ProcessPoolExecutor(max_workers=max(1, len(chunks))) as ex:
        for ch, recs in zip(chunks, ex.map(_render_rgbd_chunk, [(tuple(names), ch, width, height) for ch in chunks])):
            for (i, c), rec in zip(ch, recs):
                out[i, c - cam_lo] = rec
    return out


def triangle_indices(total: int, unique: int) -> np.ndarray:
    period = 2 * (unique - 1)
    k = np.arange(total) % period
    return np.where(k < unique, k, period - k)


# ---- algorithmic bytes --------------------------------------------------------
def frame_bytes(W: int, H: int, K: int, n_img: int = 2, n_pairs: int = 1, channels: int = 1, matchings: int = 2) -> int:
    """SURVEY.md §8d compulsory bytes per synced frame: read the images, write keypoints (12 B) and
    descriptors (32 B), write the match records (8 B per keypoint, for the stereo and the temporal
    matching of each pair).  C2: 2 * (256,000 + 88,000) + 2 * 16,000 = 720,000 B; the C3 rig frame
    is 4x that.  RGB-D (C5): one image of 5 bytes per pixel (BGR + u16 depth), temporal matching only."""
    return n_img * (W * H * channels + K * (12 + 32)) + matchings * n_pairs * K * 8


def kernel_bytes(name: str, B: int, h, cfg, maps_identity: bool, n_img_per_frame: int = 2) -> float:
    """Algorithmic (compulsory) HBM bytes of one launch of a kernel over B frames."""
    W, H, K = h.width, h.height, cfg.n_features
    imgs = n_img_per_frame * B
    pairs = imgs // 2
    pyr = sum(w * hh for w, hh in h.level_wh)
    if name == "rectify_pyramid":
        maps = 0 if maps_identity else n_img_per_frame * W * H * 8
        return imgs * (W * H + pyr) + maps
    if name == "detect":
        return imgs * (pyr + pyr)          # read the levels, write the smoothed levels
    if name == "select":
        return imgs * K * 8                # write keypoints (candidate reads are data-dependent)
    if name == "describe":
        return imgs * K * (8 + 32)         # read keypoints, write descriptors
    if name == "match":
        return pairs * 2 * (2 * K * 32 + K * 8)  # two matchings: read query+train descriptors, write best/second
    if name == "match_refine":
        return pairs * 2 * K * (8 + 16)
    if name == "pose":
        return pairs * K * (4 + 16 + 8 * 8)
    if name == "chain":
        return pairs * 68 * 8
    return 0.0


# ---- CPU baseline (the oracle on the host cores) -------------------------------------------------
def affinity_cpus() -> int:
    """CPUs in this process's affinity mask."""
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def cpu_share() -> int:
    """The host CPUs one GPU's job gets on the GPU pool (16; TSLAM_CPU_SHARE): the box exposes the
    whole node's cores (256 on the MI355X nodes) to every job, and its rules size worker pools to
    this share."""
    return max(1, int(os.environ.get("TSLAM_CPU_SHARE", "16")))


def usable_cpus() -> int:
    """CPUs this process may use: the affinity mask, capped at the per-GPU share."""
    return max(1, min(affinity_cpus(), cpu_share()))


def cpu_model() -> str:
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.startswith("Model name:"):
                return line.split(":", 1)[1].strip()
    except Exception:
        pass
    return "unknown"


def _oracle_worker(args):
    """One CPU process: the NumPy oracle tracking its contiguous frame chunk (replayed) for budget_s."""
    frames, rect_d, cfg_d, budget_s = args
    if cfg_d.get("rgbd"):
        return _oracle_worker_rgbd(args)
    from oracle import numpy_slam as O
    from thor_slam_amd.params import HipSlamConfig

    cfg = HipSlamConfig(**cfg_d)
    if isinstance(rect_d, list):   # a rig: one tracker per pair + the rig pose
        from oracle.numpy_rig import rig_pose

        rects, E = rect_d
        trks = [O.OracleTracker(cfg, r) for r in rects]
        n = 0
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < budget_s:
            i = n % len(frames)
            outs = [trk.step(frames[i, 2 * q], frames[i, 2 * q + 1]) for q, trk in enumerate(trks)]
            if n:
                rig_pose([{"status": o["status"], "T": o["T"], "corr": o.get("corr"),
                           "intr": (r["fx"], r["fy"], r["cx"], r["cy"])} for o, r in zip(outs, rects)], E, cfg)
            n += 1
        return n, time.perf_counter() - t0
    # one stereo pair: the CPU SlamEngine (oracle/numpy_engine.py, BASELINE configs[0]) through the
    # reference's loop (run_slam.py:299-328): a CameraRig replaying the chunk, initialize with the
    # rig's calibration, process_frames per synchronised set (sets built before timing)
    from oracle.numpy_engine import NumpySlamEngine
    from thor_slam_amd.camera.rig import CameraRig
    from thor_slam_amd.synthetic import CachedStereoSource

    src = CachedStereoSource(np.asarray(frames), width=frames.shape[-1], height=frames.shape[-2],
                             n_frames=len(frames))
    rig = CameraRig([src])
    rig.start()
    sets = [rig.get_synchronized_frames() for _ in range(256)]
    eng = NumpySlamEngine(num_cameras=2, config=cfg)
    eng.initialize(rig.calibration)
    n = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < budget_s:
        eng.process_frames(sets[n % len(sets)])
        eng.results.clear()   # the per-frame records are for tests
        n += 1
    return n, time.perf_counter() - t0


def _oracle_worker_rgbd(args):
    frames, rect_d, cfg_d, budget_s = args   # frames: (n, P, H, W, 3) BGR and (n, P, H, W) depth
    from oracle import numpy_slam as O
    from oracle.numpy_rig import rig_pose
    from thor_slam_amd.params import HipSlamConfig

    bgr, depth = frames
    cfg = HipSlamConfig(**cfg_d)
    rects, E = rect_d
    trks = [O.OracleTracker(cfg, r) for r in rects]
    n = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < budget_s:
        i = n % len(bgr)
        outs = [trk.step_rgbd(bgr[i, q], depth[i, q]) for q, trk in enumerate(trks)]
        if n and len(rects) > 1:
            rig_pose([{"status": o["status"], "T": o["T"], "corr": o.get("corr"),
                       "intr": (r["fx"], r["fy"], r["cx"], r["cy"])} for o, r in zip(outs, rects)], E, cfg)
        n += 1
    return n, time.perf_counter() - t0


def _rect_dict(r) -> dict:
    return dict(fx=r.fx, fy=r.fy, cx=r.cx, cy=r.cy, baseline=r.baseline, map_l=r.map_left, map_r=r.map_right)


def _run_oracle(parts: list, rect_d, cfg_d: dict, budget_s: float) -> tuple[int, float]:
    if len(parts) == 1:
        results = [_oracle_worker((parts[0], rect_d, cfg_d, budget_s))]
    else:
        with ProcessPoolExecutor(max_workers=len(parts)) as ex:
            results = list(ex.map(_oracle_worker, [(pt, rect_d, cfg_d, budget_s) for pt in parts]))
    return sum(r[0] for r in results), max(r[1] for r in results)


def cpu_baseline(frames, rect_d, cfg, budget_s: float, procs: int, what: str) -> dict:
    """The NumPy oracle on the host: `procs` processes, each tracking a contiguous chunk of the same
    frames (relative-pose work is independent per frame pair), and one process alone.
    `frames` is an array [n][...] or a (bgr, depth) pair for RGB-D."""
    import dataclasses

    cfg_d = dataclasses.asdict(cfg)

    def split(k):
        if isinstance(frames, tuple):
            return [tuple(z) for z in zip(*(np.array_split(a, k) for a in frames)) if len(z[0])]
        return [c for c in np.array_split(frames, k) if len(c)]

    parts = split(procs)
    n, wall = _run_oracle(parts, rect_d, cfg_d, budget_s)
    n1, wall1 = _run_oracle(split(1), rect_d, cfg_d, max(3.0, budget_s / 2))
    node = os.cpu_count() or 1
    rate = n / wall
    return {"value": rate, "unit": "frames/s", "cores": len(parts), "kind": "port",
            "sample": f"{n} {what} ({len(parts)} process(es) x {budget_s:.0f} s, each replaying a contiguous chunk), "
                      + ("NumpySlamEngine.process_frames (oracle/numpy_engine.py: the NumPy CPU SlamEngine of "
                         "BASELINE configs[0], through CameraRig sets as run_slam.py:299-328; this config's "
                         "loop closure / IMU / BA settings)" if not isinstance(rect_d, list) and not cfg.rgbd
                         else "NumPy oracle per pair + rig pose"),
            "single_core": {"value": n1 / wall1, "cores": 1, "sample": f"{n1} frames, 1 process x {wall1:.0f} s"},
            # the cores used are the per-GPU share of the node (pool rule: worker pools sized to
            # it); the whole node's figure is the linear extrapolation of the measured per-process
            # rate (frames are independent), stated as such
            "per_gpu_share": {"cores": len(parts), "value": rate},
            "node": {"cores": node, "affinity_cpus": affinity_cpus(), "value_extrapolated": rate / len(parts) * node,
                     "method": "measured per-process rate x node cores (not run: the pool caps a job at its share)"},
            "cpu_model": cpu_model()}


# the synthetic room (8 x 8 x 3 m, FLU) in the tracking world (rect-left camera of frame 0, RDF):
# x in [-6.9, 1.1], y in [-1.5, 1.5], z in [-4, 4] m; the volume adds 0.3-0.5 m around it
TSDF_ORIGIN = (-7.2, -1.8, -4.4)
TSDF_DIMS = (176, 72, 176)


def tsdf_report(h, us: float, B: int, width: int, height: int) -> dict:
    """k_tsdf_integrate of one batch with the colour layer: voxel (tsdf, weight) and (R, G, B,
    colour weight) read-modify-write once per launch (16 + 32 B per voxel) + the batch's depth and
    BGR images read once; the voxel-frame updates (the per-voxel projection work) beside it."""
    t, w = h.tsdf_read()
    nv = int(np.prod(TSDF_DIMS))
    observed = int((w > 0).sum())
    alg = nv * 16 + nv * 32 + B * width * height * 5   # + the colour layer (RGB + weight f32) and BGR images
    return {"kernel": "k_tsdf_integrate", "volume_voxels": nv, "voxel_size_m": 0.05, "truncation_voxels": 4,
            "frames_per_launch": B, "avg_launch_us": us, "observed_voxels": observed,
            "voxel_frame_updates_per_s": nv * B / (us * 1e-6),
            "roofline": {"bound": "hbm", "achieved": alg / (us * 1e-6) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": alg / (us * 1e-6) / 1e9 / HBM_PEAK_GBS, "algorithmic_bytes_per_launch": alg}}


_MASKED_STREAMS: list = []   # (hip library, hipStream_t) created by cu_masked_stream


def destroy_masked_streams() -> None:
    """hipStreamDestroy every stream cu_masked_stream created, after the device is idle and torch's
    current stream is back on the default one.  Streams left to the process exit were torn down by
    the HIP runtime's static destructors after rocprofv3's tool finalisation, which segfaulted
    there (__cxa_finalize) on the C4 profile of round 5."""
    import torch

    if not _MASKED_STREAMS:
        return
    torch.cuda.synchronize()
    torch.cuda.set_stream(torch.cuda.default_stream())
    while _MASKED_STREAMS:
        hip, st = _MASKED_STREAMS.pop()
        rc = hip.hipStreamDestroy(st)
        if rc != 0:
            raise RuntimeError(f"hipStreamDestroy failed ({rc})")


def cu_masked_stream(dev_index: int, reserve: int, priority: int, cus: list | None = None):
    """A torch stream whose kernels may use every CU but the last `reserve`, or only the CUs `cus`
    (hipExtStreamCreateWithCUMask); destroyed by destroy_masked_streams."""
    import ctypes

    import torch

    hip = ctypes.CDLL("libamdhip64.so")
    n_cu = torch.cuda.get_device_properties(dev_index).multi_processor_count
    words = (n_cu + 31) // 32
    mask = (ctypes.c_uint32 * words)()
    for cu in (range(n_cu - reserve) if cus is None else cus):
        mask[cu // 32] |= 1 << (cu % 32)
    st = ctypes.c_void_p()
    torch.cuda.set_device(dev_index)
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(st), ctypes.c_uint32(words), mask)
    if rc != 0:
        raise RuntimeError(f"hipExtStreamCreateWithCUMask failed ({rc})")
    hip.hipStreamDestroy.argtypes = [ctypes.c_void_p]
    _MASKED_STREAMS.append((hip, st.value))
    if priority:
        pass   # CU-masked streams take the default priority
    return torch.cuda.ExternalStream(st.value, device=torch.device("cuda", dev_index))


def dense_outputs_report(h, reps: int = 10) -> dict:
    """The dense-map outputs of the integrated volume (k_dense.hip): marching-cubes extraction
    (count + scan + one 8-byte count read back + emit) and the capped ESDF (sites, three window
    passes, finish), wall-clock per call after a synchronise, averaged over `reps` calls."""
    import ctypes

    import torch

    nv = int(np.prod(TSDF_DIMS))
    n = ctypes.c_int64()
    out = {}
    for name, call in (("mesh_extract", lambda: h.lib.tslam_mesh_extract(h.h, 1e-4, ctypes.byref(n), None)),
                       ("esdf", lambda: h.lib.tslam_esdf_compute(h.h, 2.0, 1.0, 1e-4, None))):
        call()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            call()
        torch.cuda.synchronize()
        out[name + "_us"] = (time.perf_counter() - t0) / reps * 1e6
    # ESDF: tsdf + weight read once and the f32 field written (12 B per voxel) — the rest is cache
    alg = nv * 12
    out.update({"triangles": int(n.value), "esdf_max_distance_m": 2.0, "esdf_window_voxels": 40,
                "esdf_voxels_per_s": nv / (out["esdf_us"] * 1e-6),
                "esdf_roofline": {"bound": "hbm", "achieved": alg / (out["esdf_us"] * 1e-6) / 1e9, "peak": HBM_PEAK_GBS,
                                  "unit": "GB/s", "frac": alg / (out["esdf_us"] * 1e-6) / 1e9 / HBM_PEAK_GBS,
                                  "algorithmic_bytes_per_call": alg}})
    return out


def pmc_traffic(args, dom: str, per_kernel_us: dict, B: int) -> tuple:
    """roofline.traffic (and the VALU-issue roofline) of the dominant kernel from the committed PMC
    summary (tools/pmc_summary.py) when its batch and config match this run."""
    pmc_path = Path(args.pmc)
    if not pmc_path.exists():
        return None, None, None
    pmc = json.loads(pmc_path.read_text())
    kern = pmc.get("kernels", {}).get(KERNEL_SYMBOL.get(dom, ""), None)
    if kern is None or pmc.get("batch_frames") != B or pmc.get("config", "c2") != args.config:
        return None, None, None
    valu = None
    if kern.get("valu_insts_per_launch"):
        # the path is integer-VALU bound: wave64 VALU instructions per launch
        # (PMC SQ_INSTS_VALU) / the same event-timed duration, against the issue peak
        rate = kern["valu_insts_per_launch"] / (per_kernel_us[dom] * 1e-6)
        valu = {"bound": "valu", "achieved": rate / 1e12, "peak": VALU_PEAK_WINST / 1e12,
                "unit": "T wave-instructions/s", "frac": rate / VALU_PEAK_WINST,
                "insts_per_launch": kern["valu_insts_per_launch"]}
    return kern["hbm_bytes_per_launch"], valu, kern.get("traffic_note")


# ---- the drop-in boundary (SlamEngine.process_frames on host frame sets) ----------------------
class _ReplaySource:
    """A CameraSource replaying pre-rendered [left, right] frames (triangle wave) at 30 fps
    timestamps: the CameraRig input of the boundary leg without per-frame rendering."""

    def __init__(self, name, frames, intr, extr):
        self._name, self.frames, self.intr, self.extr = name, frames, intr, extr
        self.i = 0

    @property
    def name(self):
        return self._name

    def start(self):
        pass

    def stop(self):
        pass

    def get_latest_frames(self):
        from thor_slam_amd.camera.types import CameraFrame

        k = triangle_indices(self.i + 1, len(self.frames))[-1]
        ts = 1000.0 + self.i / 30.0
        self.i += 1
        return [CameraFrame(image=self.frames[k, c], timestamp=ts, sequence_num=self.i, camera_name=f"{self._name}_{c}")
                for c in (0, 1)]

    def try_get_latest_frames(self):
        return self.get_latest_frames()

    def get_intrinsics(self):
        return self.intr

    def get_extrinsics(self):
        return self.extr

    def get_sensor_extrinsics(self):
        return None

    def get_timestamped_sensor_data(self):
        return None, None

    def try_get_timestamped_sensor_data(self):
        return None, None

    @property
    def has_sensor_data(self):
        return False


def boundary_bench(uniq: np.ndarray, src, n_frames: int, batch_sizes=(1, 64)) -> dict:
    """HipSlamEngine.process_frames timed over `n_frames` SynchronizedFrameSets produced by the
    CameraRig from host numpy frames (the reference's loop, scripts/run_slam.py:314-328), per
    engine batch size; frame sets are built before timing (the camera is not what is measured)."""
    from thor_slam_amd.camera.rig import CameraRig
    from thor_slam_amd.params import HipSlamConfig
    from thor_slam_amd.slam.hip_engine import HipSlamEngine

    rep = _ReplaySource(src.name, uniq, src.get_intrinsics(), src.get_extrinsics())
    rig = CameraRig([rep])
    rig.start()
    sets = []
    while len(sets) < n_frames:
        s = rig.get_synchronized_frames()
        if s is not None:
            sets.append(s)
    out = {"frames": n_frames, "image_bytes_per_frame": int(uniq[0].nbytes)}
    for b in batch_sizes:
        eng = HipSlamEngine(num_cameras=2, config=HipSlamConfig(batch_size=b, enable_loop_closure=False))
        eng.initialize(rig.calibration)
        for s in sets[:2 * b + 8]:   # warm-up
            eng.process_frames(s)
        eng.flush()
        eng.reset()
        t0 = time.perf_counter()
        for s in sets:
            eng.process_frames(s)
        eng.flush()
        dt = time.perf_counter() - t0
        st = eng.get_tracking_state()
        eng.shutdown()
        out[f"fps_b{b}"] = n_frames / dt
        out[f"ingress_GBps_b{b}"] = n_frames * uniq[0].nbytes / dt / 1e9
        out[f"state_b{b}"] = st.name
    return out


# ---- the reference's default drop-in path ----------------------------------
LAP = 240          # one full turn of the 45 deg/s circle at 30 fps: the trajectory repeats
C3_NAMES = ("192.168.2.21", "192.168.2.22", "192.168.2.23", "192.168.2.25")   # run_slam.py:45-50


def _lap_sources(names, frames=None):
    """Stereo sources on the bracket joints along one repeating turn (IMU on the first, with the
    noise of an OAK-class MEMS IMU); with `frames` ({name: [LAP][2][H][W]}) they replay them."""
    from thor_slam_amd.synthetic import CachedStereoSource, RoomScene, SyntheticStereoSource, circle_trajectory

    joints = json.loads(JOINTS.read_text())
    scene, traj = RoomScene(seed=0), circle_trajectory(LAP, yaw_rate_deg=45.0)
    out = []
    for k, nm in enumerate(names):
        kw = dict(name=nm, scene=scene, trajectory=traj, rig_T_source=np.array(joints[nm]), seed=k, imu=(k == 0),
                  gyro_noise=1e-4, accel_noise=0.01)
        out.append(CachedStereoSource(frames[nm], **kw) if frames is not None else SyntheticStereoSource(**kw))
    return out


def _render_lap_chunk(args):
    names, items = args   # items: (source index, frame, camera)
    srcs = _lap_sources(names)
    return [srcs[q].render_image(i, c) for q, i, c in items]


def default_config_bench(kind: str, n_frames: int, workers: int) -> dict:
    """SlamEngine.process_frames exactly as the reference deploys it after the two-line swap
    (scripts/run_slam.py:299-300): HipSlamEngine(num_cameras=N) + initialize(rig.calibration), no
    config — batch 1, loop closure on (SlamConfig.enable_loop_closure, interface.py:156), IMU fusion
    on because the rig carries the IMU (Makefile:81, run_slam.py:249-283).  The rig replays one
    rendered turn of a 45 deg/s circle with its IMU samples, so from the second lap on every
    keyframe finds the previous lap: the worst case for loop closure (a search, a verification and
    a span solve per keyframe).  Frame sets are built before timing."""
    from thor_slam_amd.camera import CameraRig, Extrinsics
    from thor_slam_amd.camera.types import IMUExtrinsics
    from thor_slam_amd.slam.hip_engine import HipSlamEngine
    from thor_slam_amd.synthetic import DRB_TO_RDF

    names = C3_NAMES if kind == "c3" else C3_NAMES[:1]
    t0 = time.perf_counter()
    items = [(q, i, c) for q in range(len(names)) for i in range(LAP) for c in (0, 1)]
    chunks = [items[k::workers] for k in range(workers) if items[k::workers]]
    frames = {nm: np.empty((LAP, 2, 400, 640), np.uint8) for nm in names}
    with ProcessPoolExecutor(max_workers=max(1, len(chunks))) as ex:
        for ch, imgs in zip(chunks, ex.map(_render_lap_chunk, [(names, ch) for ch in chunks])):
            for (q, i, c), img in zip(ch, imgs):
                frames[names[q]][i, c] = img
    t_render = time.perf_counter() - t0
    joints = json.loads(JOINTS.read_text())
    srcs = _lap_sources(names, frames)
    base_T_imu = np.array(joints[names[0]]) @ DRB_TO_RDF
    rig = CameraRig(srcs, rig_extrinsics={nm: Extrinsics.from_4x4_matrix(np.array(joints[nm])) for nm in names},
                    imu_source=names[0], imu_extrinsics=IMUExtrinsics(names[0], Extrinsics.from_4x4_matrix(base_T_imu)))
    rig.start()
    warm = 64
    sets = []
    while len(sets) < warm + n_frames:
        fs = rig.get_synchronized_frames()
        if fs is not None:
            sets.append(fs)
    out = {"cameras": 2 * len(names), "frames": n_frames, "render_s": t_render}
    for mode in ("default", "sync"):
        from thor_slam_amd.params import HipSlamConfig

        eng = HipSlamEngine(num_cameras=2 * len(names))
        if mode == "default":
            eng.initialize(rig.calibration)   # the reference's call: no config
        else:   # the same with every batch waited for (the round-4 behaviour of this configuration)
            eng.initialize(rig.calibration, HipSlamConfig(num_cameras=2 * len(names), sync=True))
        cfg = eng._config
        for fs in sets[:warm]:   # kernels, loop jobs and the pose-graph scratch warm up
            eng.process_frames(fs)
        eng.settle()
        eng.reset()
        t1 = time.perf_counter()
        for fs in sets[warm:]:
            eng.process_frames(fs)
        eng.flush()
        dt = time.perf_counter() - t1
        lp = eng._loop
        rec = {"fps": n_frames / dt, "batch_size": cfg.batch_size, "loop_closure": lp is not None,
               "imu_fusion": eng._imu is not None, "imu_prior_lag": cfg.imu_prior_lag,
               "loop_latency_frames": cfg.loop_latency, "asynchronous": bool(eng._async),
               "keyframes": len(lp.frames) if lp is not None else 0,
               "loops_closed": len(lp.loops) if lp is not None else 0,
               "state": eng.get_tracking_state().name}
        eng.shutdown()
        if mode == "default":
            out.update(rec)
        else:
            out["sync_fps"] = rec["fps"]
    return out


# ---- single handle (N = 1, and c5 replicas) ---------------------------------------------------
def run_single(args, world: int, rank: int, dev_index: int) -> dict:
    import torch
    import torch.distributed as dist

    from thor_slam_amd._lib import KERNELS, Handle
    from thor_slam_amd.calib import extract_cameras, stereo_pairs, stereo_rectify
    from thor_slam_amd.camera.rig import CameraRig
    from thor_slam_amd.params import HipSlamConfig
    from thor_slam_amd.synthetic import SyntheticStereoSource

    c3, c4, c5 = args.config == "c3", args.config == "c4", args.config == "c5"
    width, height = (1280, 800) if c4 else (1280, 720) if c5 else (640, 400)
    cfg = (HipSlamConfig(n_features=4000, ba_window=10, ba_kf_interval=5, ba_iters=5) if c4 else
           HipSlamConfig(rgbd=True) if c5 else HipSlamConfig())
    B = args.batch or (50 if c4 else C5_BATCH if c5 else C3_BATCH if c3 else C2_BATCH)
    # C2 replays 1,024 distinct frames (512 MB of input, twice the 256 MB MALL, so the input reads
    # are not cache hits; 48 replayed ones ran 2 % faster, gpurun_out r5bl); the others 48 / 24
    args.unique = args.unique or (24 if (c4 or c5) else 48 if c3 else C2_UNIQUE)
    workers = max(1, min(16, usable_cpus(), args.unique * (8 if c3 else 1)))
    t_r = time.perf_counter()
    E = None
    src = None
    if c5:   # the 4-camera RGB-D rig, whole on this GPU: records [n][4][5HW]
        _, cams, pairs, rects, E = rgbd_rig_setup(RIG_SOURCES, width, height)
        uniq = render_rgbd_rig_frames(RIG_SOURCES, args.unique, 0, len(rects), workers, width, height)
    elif c3:
        _, cams, pairs, rects, E = rig_setup(RIG_SOURCES, width, height)
        uniq = render_rig_frames(RIG_SOURCES, args.unique, 0, 2 * len(rects), workers, width, height)
    else:
        src = SyntheticStereoSource(seed=rank, n_frames=args.unique, width=width, height=height)
        cams = extract_cameras(CameraRig([src]).calibration, 2)
        (li, ri), = stereo_pairs(cams)
        rects = [stereo_rectify(cams[li], cams[ri])]
        uniq = render_frames(rank, args.unique, workers, width, height)
    t_render = time.perf_counter() - t_r
    P = len(rects)
    rect = rects[0]
    n_img = uniq.shape[1] if not c5 else 1

    total = (args.warmup + args.steps) * B
    if c5:
        # one batch in HBM, replayed every step: the batch spans whole periods of the triangle
        # wave, so consecutive batches continue it seamlessly (4.6 MB per record keeps the resident
        # input at one batch instead of (warmup + steps) of them)
        period = 2 * (args.unique - 1)
        if B % period:
            raise SystemExit(f"--config c5 needs --batch a multiple of {period} (2 x (unique - 1))")
        total = B
    # the triangle wave repeats every 2 (unique - 1) frames, so one period + one batch of it in HBM
    # holds every batch: step s starts at (s B) mod period (the resident input stays ~2 GB at C2
    # whatever --steps is, and the frame sequence stays continuous past the timed region)
    period = max(1, 2 * (args.unique - 1))
    wrap = not c5 and total > period + B
    if wrap:
        total = period + B
    idx = torch.from_numpy(triangle_indices(total, args.unique)).cuda()
    seq = torch.from_numpy(uniq).cuda().index_select(0, idx).contiguous()  # [total, C, H, W] (c5: [B, 4, 5HW]) in HBM
    # the outlier steps after the timed region replay the resident batches
    step_base = (lambda s: 0) if c5 else (lambda s: (s * B) % period) if wrap else (lambda s: (s % (args.warmup + args.steps)) * B)
    h = Handle(rects, cfg, max_batch=B, device=dev_index)
    if P > 1:
        h.set_rig(E)
    # the front stream (rectify .. describe) is the critical path of the pipelined step: with
    # --front-priority 1 it is a high-priority stream, so the back kernels fill the gaps around it
    stream = (torch.cuda.Stream(priority=-1) if args.front_priority and args.pipeline else torch.cuda.current_stream())
    if args.front_cu_reserve < 0:
        args.front_cu_reserve = 96 if c4 else 0
    masked = c4 and args.front_cu_reserve > 0 and args.pipeline
    if masked:   # C4: the front / back kernels kept off the last CUs, which stay free for the BA chain
        stream = cu_masked_stream(dev_index, args.front_cu_reserve, -1 if args.front_priority else 0)
    torch.cuda.set_stream(stream)
    sp = stream.cuda_stream
    # the rig pose runs before the chains (KERNEL_CHAIN chains the pairs and the rig in one launch)
    kern = [k for k in KERNELS if k != "chain"] + (["rig"] if P > 1 else []) + ["chain"]
    names = kern + (["local_ba"] if c4 else []) + (["tsdf"] if c5 and args.tsdf else [])
    if c5 and args.tsdf:
        h.tsdf_color(True)   # nvblox's colour layer with the TSDF (the engine's default)
        h.tsdf_init(TSDF_ORIGIN, TSDF_DIMS, 0.05, 4.0, 10.0, 100.0)
    BACK = {"match", "match_refine", "pose", "chain", "rig"}
    # two streams: the front kernels (rectify .. describe) of batch s + 1 overlap the back kernels
    # (match .. chain) of batch s; the library orders batch s's back after its front and batch s's
    # front after the back of batch s - 2 (ring slots)
    bstream = (cu_masked_stream(dev_index, args.front_cu_reserve, 0) if masked else torch.cuda.Stream()) if args.pipeline else stream
    if args.back_cu and args.pipeline and not masked:   # experiment: the back kernels on N CUs spread over the chip
        n_cu = torch.cuda.get_device_properties(dev_index).multi_processor_count
        back_set = [i * n_cu // args.back_cu for i in range(args.back_cu)]
        bstream = cu_masked_stream(dev_index, 0, 0, back_set)
        if args.split_cu:   # and the front kernels on the other CUs (disjoint)
            stream = cu_masked_stream(dev_index, 0, 0, sorted(set(range(n_cu)) - set(back_set)))
            torch.cuda.set_stream(stream)
            sp = stream.cuda_stream
    bsp = bstream.cuda_stream
    back_done = [torch.cuda.Event(), torch.cuda.Event()]
    back_issued = [False, False]
    # C4: local BA runs on a third stream, overlapping the next batches
    ba_stream = torch.cuda.Stream(priority=-1 if args.ba_priority else 0) if c4 else None
    if c4 and args.pipeline and args.ba_defer:
        # the BA's ~160 host launches per batch enqueued after the next batch's front stages
        # (tslam_ba_defer), so the front end of batch s+1 overlaps the BA of batch s on the GPU
        h.ba_defer(True)
    if c4 and args.ba_cus > 0:   # experiment: the BA chain only on the last N CUs (the front / back keep off them)
        n_cu = torch.cuda.get_device_properties(dev_index).multi_processor_count
        ba_stream = cu_masked_stream(dev_index, 0, 0, list(range(n_cu - args.ba_cus, n_cu)))
    ba_done = [torch.cuda.Event(), torch.cuda.Event()] if c4 else None
    ba_issued = [False, False]
    ba_host = [0.0, 0]   # C4: host seconds spent enqueuing the BA stage, calls

    # kernels bracketed by HIP events inside the timed steps: every event pair is a marker on the
    # GPU timeline, so by default only the dominant kernel's (detect; the roofline's live launch
    # time) — the other kernels' durations come from the isolated runs after the timed region
    timed_all = args.kernel_events == "all"
    timed_set = set(args.kernel_events.split(",")) if not timed_all else set(names)

    def run(k: str, st) -> None:
        if k == "rig":
            h.run_rig(st.cuda_stream)
        else:
            h.run_kernel(k, st.cuda_stream)

    def step(s: int, evs=None, outliers: int = 0) -> None:
        # one batch = every kernel of the hot path; in the timed steps each kernel is bracketed by
        # a pair of HIP events on the stream it runs on (the per-kernel durations below).
        # `outliers` > 0: that percentage of the refined temporal positions is moved 8-40 px before
        # the pose kernels (tslam_perturb_temporal, a benchmark hook) — RANSAC on hard data
        h.begin_batch(seq[step_base(s)].data_ptr(), B)
        # the waits the library would insert, made here so the events time kernels, not waits
        if c4 and ba_issued[s % 2]:
            stream.wait_event(ba_done[s % 2])
        if bstream is not stream and back_issued[s % 2]:
            stream.wait_event(back_done[s % 2])
        first_back = True
        for i, k in enumerate(names):
            if k == "tsdf":
                continue
            if k == "local_ba":
                ba_stream.wait_stream(bstream)
                if evs is not None:
                    evs[i][0].record(ba_stream)
                t_ba = time.perf_counter()
                h.run_stage("ba", ba_stream.cuda_stream)
                ba_host[0] += time.perf_counter() - t_ba
                ba_host[1] += 1
                ba_done[s % 2].record(ba_stream)
                ba_issued[s % 2] = True
                if evs is not None:
                    evs[i][1].record(ba_stream)
                continue
            st = bstream if k in BACK else stream
            if k in BACK and first_back and bstream is not stream:
                bstream.wait_stream(stream)
                first_back = False
            timed = evs is not None and (timed_all or k in timed_set or (outliers and k == "pose"))
            if outliers and k == "pose":
                h.perturb_temporal(outliers, seed=s, stream=st.cuda_stream)
            if timed:
                evs[i][0].record(st)
            run(k, st)
            if timed:
                evs[i][1].record(st)
        if bstream is not stream:
            back_done[s % 2].record(bstream)
            back_issued[s % 2] = True
        h.end_batch()
        if "tsdf" in names:   # the batch's depth into the volume, with its device-resident poses
            i = names.index("tsdf")
            if evs is not None:
                evs[i][0].record(bstream)
            base = seq[step_base(s)].data_ptr()
            h.tsdf_integrate_rgbd(base, base + 3 * width * height, 5 * width * height * P, B, first_frame=s * B,
                                  stream=bsp)
            if evs is not None:
                evs[i][1].record(bstream)

    events = [[(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in names]
              for _ in range(args.steps)]
    for s in range(args.warmup):
        step(s)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(args.warmup + k, events[k])
    t_issue = time.perf_counter() - t0   # host time to issue the steps (launches are asynchronous)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    res = h.read_poses(B)
    ok_frac = float(np.mean(res["stats"][:, :, 0] == 0))
    rig_ok = float(np.mean(h.read_rig_poses(B)["stats"][:, 0] == 0)) if P > 1 else None

    # ---- the same kernels run alone (after the timed region, one stream, 3 batches): under the
    # two-stream pipeline a kernel shares the GPU with the other stream's kernels, so its timed
    # duration above includes that sharing; these isolated durations are the kernel's own speed
    iso_us = {k: 0.0 for k in kern}
    n_iso = 3
    torch.cuda.synchronize()
    for r in range(n_iso):
        s_iso = r % (args.warmup + args.steps)   # replayed input: only the durations are used
        h.begin_batch(seq[step_base(s_iso)].data_ptr(), B)
        prs = []
        for k in kern:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            run(k, stream)
            e1.record(stream)
            prs.append((k, e0, e1))
        h.end_batch()
        torch.cuda.synchronize()
        for k, e0, e1 in prs:
            iso_us[k] += e0.elapsed_time(e1) * 1e3 / n_iso

    # ---- the pose stage on hard data: the same pipelined steps with
    # --outliers % of every frame's refined temporal positions made outliers before the pose
    # kernels, so the bounded RANSAC scoring cannot end at the first correct root
    pose_outliers = None
    if args.outliers > 0 and args.outlier_steps > 0 and not (c4 or c5):
        ev_o = [[(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in names]
                for _ in range(args.outlier_steps)]
        base_s = args.warmup + args.steps
        step(base_s, outliers=args.outliers)   # warm-up (the learnt FAST threshold is unaffected)
        torch.cuda.synchronize()
        t_o = time.perf_counter()
        for k in range(args.outlier_steps):
            step(base_s + 1 + k, ev_o[k], outliers=args.outliers)
        torch.cuda.synchronize()
        el_o = time.perf_counter() - t_o
        res_o = h.read_poses(B)
        st_o = res_o["stats"][:, :, :]
        ip = names.index("pose")
        pose_pipe = sum(e[ip][0].elapsed_time(e[ip][1]) for e in ev_o) * 1e3 / args.outlier_steps
        # the pose kernels alone on one stream, on a perturbed batch (3 batches)
        iso_o = 0.0
        for r in range(3):
            h.begin_batch(seq[step_base(r)].data_ptr(), B)
            for k in kern:
                if k == "pose":
                    h.perturb_temporal(args.outliers, seed=1000 + r, stream=sp)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(stream)
                    run(k, stream)
                    e1.record(stream)
                elif k not in ("rig", "chain"):
                    run(k, stream)
            h.end_batch()
            torch.cuda.synchronize()
            iso_o += e0.elapsed_time(e1) * 1e3 / 3
        ok_o = st_o[:, :, 0] == 0
        inl = np.where(ok_o, st_o[:, :, 2] / np.maximum(st_o[:, :, 1], 1), np.nan)
        pose_outliers = {
            "outlier_pct": args.outliers, "steps": args.outlier_steps,
            "ms_per_step": el_o / args.outlier_steps * 1e3,
            "frames_per_s": args.outlier_steps * B / el_o,
            "pose_us_pipelined": pose_pipe, "pose_us_isolated": iso_o,
            "clean_pose_us_isolated": iso_us["pose"],
            "tracking_ok_fraction_last_batch": float(np.mean(ok_o)),
            "inlier_fraction_mean": float(np.nanmean(inl)) if np.isfinite(inl).any() else None,
            "method": "tslam_perturb_temporal (benchmark hook) between match_refine and pose: that share of every "
                      "frame's refined temporal positions moved 8-40 px per axis; same pipelined steps and kernels",
        }

    # ---- per-kernel durations of the timed launches (HIP events on the launch stream) ----------
    per_kernel_us = {}
    for evs in events:
        for i, k in enumerate(names):
            if timed_all or k in timed_set:
                per_kernel_us[k] = per_kernel_us.get(k, 0.0) + evs[i][0].elapsed_time(evs[i][1]) * 1e3 / args.steps  # us
    unit_bytes = (frame_bytes(rect.width, rect.height, cfg.n_features, n_img=P, n_pairs=P, channels=5, matchings=1) if c5 else
                  frame_bytes(rect.width, rect.height, cfg.n_features, n_img=2 * P, n_pairs=P))
    dom_bytes = unit_bytes * B          # §8d per-frame bytes x the frames one launch processes
    # C4's MFMA kernel: back-to-back replays of k_ba_schur on the last solved window, between two
    # HIP events (per-launch events inside the timed steps would add their own gaps to the BA chain)
    schur = h.ba_replay_schur(0, 50, sp) if c4 else None
    front = {k: v for k, v in per_kernel_us.items() if k not in ("local_ba", "tsdf")}
    if not front:
        raise SystemExit("--kernel-events must name at least one front-end kernel (the roofline's live launch time)")
    dom = max(front, key=front.get)
    achieved = dom_bytes / (per_kernel_us[dom] * 1e-6) / 1e9
    mfma = None
    if schur and schur["flops"] > 0:
        avg_us, flops = schur["us"], schur["flops"]
        mfma = {"bound": "mfma", "kernel": "k_ba_schur", "achieved": flops / (avg_us * 1e-6) / 1e12,
                "peak": FP64_MFMA_PEAK_TFS, "unit": "TFLOP/s", "traffic": None, "dtype": "f64",
                "algorithmic_flops_per_launch": flops,
                "flop_count": "symmetric product C = Q^T Q: rows (rows + 1) 3L, rows = 6 n + 1 (lower triangle only)",
                "avg_launch_us": avg_us, "launches_timed": schur["reps"],
                "timing": "HIP events around back-to-back replays on the last solved window",
                # launches per step: keyframes x Gauss-Newton iterations x pairs
                "time_per_step_us": avg_us * (B // cfg.ba_kf_interval) * cfg.ba_iters * P}
        mfma["frac"] = mfma["achieved"] / mfma["peak"]
    traffic, valu, traffic_note = pmc_traffic(args, dom, per_kernel_us, B)

    # ---- B = 1 latency: one frame submitted and its pose read back -------------
    lat_ms = None
    if rank == 0 and args.latency_frames > 0:
        h1 = Handle(rects, cfg, max_batch=1, device=dev_index)
        if P > 1:
            h1.set_rig(E)
        lat = []
        for i in range(args.latency_frames + 3):
            torch.cuda.synchronize()
            ta = time.perf_counter()
            h1.submit(seq[i].data_ptr(), 1, sp)
            h1.read_poses(1)
            if i >= 3:
                lat.append((time.perf_counter() - ta) * 1e3)
        h1.close()
        lat_ms = float(np.median(lat))

    frames_total = world * args.steps * B
    roofline = {
        "bound": "hbm",
        "kernel": dom,
        "achieved": achieved,
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": achieved / HBM_PEAK_GBS,
        "traffic": traffic,
        "traffic_note": traffic_note,
        "algorithmic_bytes_per_launch": dom_bytes,
        "algorithmic_bytes_per_frame": unit_bytes,
        "frames_per_launch": B,
        "avg_launch_us": per_kernel_us[dom],
        "largest_isolated_kernel": max(iso_us, key=iso_us.get),
        "kernel_own_bytes_per_launch": None if c5 else kernel_bytes(dom, B, h, cfg, rect.is_identity, n_img),
        "end_to_end_hbm_frac": unit_bytes * (frames_total / elapsed / world) / (HBM_PEAK_GBS * 1e9),
        "valu": valu,
    }
    # the dominant kernel measured alone: the same algorithmic bytes (and PMC VALU instructions)
    # over its isolated duration
    iso = {"avg_launch_us": iso_us[dom], "achieved": dom_bytes / (iso_us[dom] * 1e-6) / 1e9}
    iso["frac"] = iso["achieved"] / HBM_PEAK_GBS
    if valu is not None:
        iso["valu_frac"] = valu["insts_per_launch"] / (iso_us[dom] * 1e-6) / VALU_PEAK_WINST
    roofline["isolated"] = iso
    if mfma is not None and mfma["time_per_step_us"] > per_kernel_us[dom]:
        roofline, front_roofline = mfma, roofline   # the Schur product is the step's dominant kernel
    else:
        front_roofline = None
    if c5:
        workload = ("C5: 4-camera RGB-D rig (brackets.urdf joints, sources of run_slam.py:45-50), 1280x720 BGR u8 + "
                    "aligned u16 mm depth per camera, on-device gray conversion, 2000 FAST/rBRIEF keypoints, 4 levels, "
                    "temporal brute-force Hamming, depth-lookup 3D points, P3P-RANSAC(128)+GN per camera, rig pose "
                    "by generalised PnP over all cameras, on one GPU")
    elif c4:
        workload = ("C4: 1x stereo pair 1280x800, 4000 FAST/rBRIEF keypoints per image, 4 levels, stereo+temporal "
                    "brute-force Hamming, P3P-RANSAC(128)+GN pose, 10-keyframe local BA (keyframe every 5 frames, "
                    "5 Gauss-Newton iterations, Schur complement on FP64 MFMA)")
    elif c3:
        workload = ("C3: 4x OAK stereo rig (8 streams, brackets.urdf joints, sources of run_slam.py:45-50) 640x400, "
                    "2000 FAST/rBRIEF keypoints per image, per-pair stereo+temporal brute-force Hamming + "
                    "P3P-RANSAC(128)+GN, rig pose by generalised PnP over all pairs, on one GPU")
    else:
        workload = ("C2: 1x stereo pair 640x400 per GPU, 2000 FAST/rBRIEF keypoints per image, 4 levels, "
                    "stereo+temporal brute-force Hamming, P3P-RANSAC(128)+GN pose")
    value = frames_total / elapsed
    out = {
        "metric": METRIC_C4 if c4 else METRIC_C5 if c5 else METRIC_C3 if c3 else METRIC,
        "value": value,
        "unit": "frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "host_issue_ms_per_step": t_issue / args.steps * 1e3,   # host time to enqueue a step
        "host_ba_issue_ms_per_call": (ba_host[0] / ba_host[1] * 1e3) if c4 and ba_host[1] else None,
        "higher_is_better": True,
        "scaling": "strong" if (c3 or c5) else "weak",
        "vs_baseline": None,
        "dtype": "u8+f64",
        "data": f"synthetic: seeded room renderer, {args.unique} distinct {width}x{height} "
                f"{'RGB-D' if c5 else 'rig' if c3 else 'stereo'} frames per rank replayed as a triangle wave, "
                f"resident in HBM before timing",
        "config": {
            "workload": workload,
            "frames_per_step": B,
            "n_features": cfg.n_features,
            "parallelism": (f"one stereo source per GPU x{world}" + (" (independent replicas)" if world > 1 else ""))
                           if not (c3 or c5) else "the whole rig on 1 GPU",
            **({"streams": "front + back kernels CU-masked off the last "
                           f"{args.front_cu_reserve} CUs, local BA on a third stream on "
                           + (f"the last {args.ba_cus} CUs only" if args.ba_cus > 0 else "every CU")} if masked else {}),
        },
        "roofline": roofline,
        "latency_b1_ms": lat_ms,
        "pose_with_outliers": pose_outliers,
        "per_kernel_us_per_batch": per_kernel_us,
        "per_kernel_us_isolated": iso_us,
        "tracking_ok_fraction_last_batch": ok_frac,
        "rig_ok_fraction_last_batch": rig_ok,
        "render_s": t_render,
    }
    if c3:
        out["stereo_pair_frames_per_s"] = value * P
    if c5:
        out["camera_frames_per_s"] = value * P
    if front_roofline is not None:
        out["front_end_roofline"] = front_roofline
    if "tsdf" in names:
        out["dense_map"] = tsdf_report(h, per_kernel_us["tsdf"], B, width, height)
        out["dense_map"]["outputs"] = dense_outputs_report(h)
    h.close()
    destroy_masked_streams()
    if rank == 0 and world == 1 and args.boundary_frames > 0 and args.config == "c2":
        out["boundary"] = boundary_bench(uniq, src, args.boundary_frames)
        if args.default_frames > 0:
            workers = usable_cpus()
            out["boundary"]["default_config"] = {
                "c2": default_config_bench("c2", args.default_frames, workers),
                "c3": default_config_bench("c3", max(args.default_frames // 2, 1), workers)}
    if rank == 0 and world == 1 and args.cpu_budget > 0:
        procs = args.cpu_procs or usable_cpus()
        if c5:
            from thor_slam_amd.rgbd import unpack_rgbd

            bgr = np.empty((len(uniq), P, height, width, 3), np.uint8)
            dep = np.empty((len(uniq), P, height, width), np.uint16)
            for i in range(len(uniq)):
                for q in range(P):
                    bgr[i, q], dep[i, q] = unpack_rgbd(uniq[i, q], width, height)
            out["cpu_baseline"] = cpu_baseline((bgr, dep), [[_rect_dict(r) for r in rects], E], cfg, args.cpu_budget,
                                               procs, f"synthetic {width}x{height} 4-camera RGB-D rig frames "
                                                      f"({len(bgr)} distinct)")
            out["cpu_baseline"]["unit"] = "rig frames/s"
        elif c3:
            out["cpu_baseline"] = cpu_baseline(uniq, [[_rect_dict(r) for r in rects], E], cfg, args.cpu_budget, procs,
                                               f"synthetic {width}x{height} 8-stream rig frames ({len(uniq)} distinct)")
            out["cpu_baseline"]["unit"] = "rig frames/s"
        else:
            out["cpu_baseline"] = cpu_baseline(uniq, _rect_dict(rect), cfg, args.cpu_budget, procs,
                                               f"synthetic {width}x{height} stereo frames ({len(uniq)} distinct)")
    return out


# ---- sharded rig (N > 1): one camera stream per GPU -------------------------------------------
def run_sharded(args, world: int, rank: int, dev_index: int) -> dict:
    """The sharded rig through the library's own driver (tslam_shard.cpp, the code the SlamEngine and
    the C-ABI ship): one process per rank over RCCL (tslam_comm_init + tslam_submit_sharded), or
    with ``--transport copy`` all ranks in this one process on one GPU (tslam_group_create, device
    copies: a rehearsal of the exchange on a one-GPU box).  ``--driver torch`` runs the
    torch.distributed test double (thor_slam_amd/shard.py: DistShardedRig) instead."""
    import torch
    import torch.distributed as dist

    from thor_slam_amd.params import HipSlamConfig
    from thor_slam_amd.shard import DistShardedRig, ShardPlan, StageTimer

    c3, c5 = args.config == "c3", args.config == "c5"
    rehearse = args.transport == "copy"
    if args.config == "c2" and world % 2:
        raise SystemExit("c2 over several GPUs shards stereo pairs' streams: --gpus must be even")
    if c5 and 4 % world:
        raise SystemExit("c5 shards the 4 RGB-D cameras: --gpus must be 1, 2 or 4")
    names = RIG_SOURCES if (c3 or c5) else RIG_SOURCES[:world // 2]
    width, height = (1280, 720) if c5 else (640, 400)
    cfg = HipSlamConfig(rgbd=True) if c5 else HipSlamConfig()
    B = args.batch or (C5_BATCH if c5 else C3_BATCH if c3 else C2_BATCH)
    args.unique = args.unique or (24 if c5 else 48 if c3 else C2_UNIQUE)
    if c5:
        _, cams, pairs, rects, E = rgbd_rig_setup(names, width, height)
        C = len(rects)
    else:
        _, cams, pairs, rects, E = rig_setup(names, width, height)
        C = 2 * len(rects)
    P = len(rects)
    plan = ShardPlan(C, world, B)
    local = list(range(world)) if rehearse else [rank]   # the ranks this process drives
    c0, c1 = (0, C) if rehearse else plan.cams(rank)
    workers = max(1, min(16, max(2, usable_cpus() // max(1, 1 if rehearse else world)), args.unique * (c1 - c0)))
    t_r = time.perf_counter()
    if c5:   # this process's cameras only; one batch resident, replayed (whole triangle-wave periods)
        uniq = render_rgbd_rig_frames(names, args.unique, c0, c1, workers, width, height)
        if B % (2 * (args.unique - 1)):
            raise SystemExit(f"--config c5 needs --batch a multiple of {2 * (args.unique - 1)}")
        total = B
    else:
        uniq = render_rig_frames(names, args.unique, c0, c1, workers, width, height)   # this process's streams only
        total = (args.warmup + args.steps) * B
    period = max(1, 2 * (args.unique - 1))
    wrap = not c5 and total > period + B   # one period + one batch of the triangle wave holds every batch
    if wrap:
        total = period + B
    t_render = time.perf_counter() - t_r
    idx = torch.from_numpy(triangle_indices(total, args.unique)).cuda()
    S = plan.streams_per_rank
    seqs = []   # per local rank: [total, S, H, W] (RGB-D: records) in HBM
    full = torch.from_numpy(uniq).cuda()
    for r in local:
        lo = (plan.cams(r)[0] - c0)
        seqs.append(full[:, lo:lo + S].index_select(0, idx).contiguous())
    del full
    batch_of = ((lambda q, s: seqs[q]) if c5 else
                (lambda q, s: seqs[q][(s * B) % period:(s * B) % period + B]) if wrap else
                (lambda q, s: seqs[q][s * B:(s + 1) * B]))
    stream = torch.cuda.current_stream()
    if args.driver == "torch":
        if rehearse:
            raise SystemExit("--transport copy rehearses the library driver (--driver library)")
        rig = DistShardedRig(rects, cfg, B, base_T_rect=E if P > 1 else None, device=dev_index, exchange=args.exchange,
                             front_priority=bool(args.front_priority))
        step = lambda s, timer=None: rig.step(batch_of(0, s), timer)   # noqa: E731
        drain = rig.drain
    else:
        from thor_slam_amd._lib import Handle, HandleGroup, comm_unique_id

        hs = [Handle(rects, cfg, max_batch=B, device=dev_index) for _ in local]
        for h in hs:
            if P > 1:
                h.set_rig(E)
        pairs = bool(args.pair_split)
        if pairs and (c5 or S != 1):
            raise SystemExit("--pair-split shards a stereo rig with one camera stream per GPU")
        if rehearse:
            grp = HandleGroup(hs, "copy")
            hs[0].shard_options(pipeline=True, pairs=pairs)
            step = lambda s, timer=None: grp.submit([batch_of(q, s).data_ptr() for q in range(world)], B,  # noqa: E731
                                                    [stream.cuda_stream] * world)
        else:
            uid = [comm_unique_id() if rank == 0 else None]
            if world > 1:
                dist.broadcast_object_list(uid, src=0)
            hs[0].comm_init(uid[0], rank, world)
            hs[0].shard_options(pipeline=True, pairs=pairs)   # batch s+1's front end beside batch s's back end
            step = lambda s, timer=None: hs[0].submit_sharded(batch_of(0, s).data_ptr(), B, stream.cuda_stream)  # noqa: E731
        drain = torch.cuda.synchronize
    for s in range(args.warmup):
        step(s)
    drain()
    if world > 1 and not rehearse:
        dist.barrier()
    torch.cuda.synchronize()
    timer = StageTimer()
    if args.driver == "library":
        hs[0].shard_options(profile=True, pipeline=True, pairs=bool(args.pair_split))
    t0 = time.perf_counter()
    for k in range(args.steps):
        s = args.warmup + k
        step(s, timer)
    drain()
    if world > 1 and not rehearse:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1 and not rehearse:
        tt = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    if args.driver == "library":
        timings = [h.shard_timing()[0] for h in hs]
        per_kernel_us = {k: max(t[k] for t in timings) for k in timings[0]}   # the slowest local rank
        per_kernel_us = {k: v for k, v in per_kernel_us.items() if v > 0.0}
        res = {"pairs": hs[0].read_poses(B)}
        if P > 1:
            res["rig"] = hs[0].read_rig_poses(B)
        sb, pr = hs[0].exchange_sizes()
        pb = hs[0].pair_block_bytes() if (c5 or args.pair_split) else 0
    else:
        res = rig.read()
        per_kernel_us = timer.mean_us()
        sb, pr = rig.rk.block, rig.rk.record
        pb = rig.rk.pblock if c5 else 0
    ok = float(np.mean(res["pairs"]["stats"][:, :, 0] == 0))
    rig_ok = float(np.mean(res["rig"]["stats"][:, 0] == 0)) if P > 1 else None
    # exchange spans (HIP events across the streams): not kernels, reported on their own
    exchange_us = {k: per_kernel_us.pop(k) for k in ("exchange_exposed", "exchange_wait", "pose_gather") if k in per_kernel_us}
    # the dominant kernel's algorithmic bytes: the §8d rig-frame bytes x the share of the rig one
    # launch covers (front kernels: S of C streams for B frames; back kernels: all streams for B/N frames)
    S = plan.streams_per_rank
    unit_bytes = (frame_bytes(width, height, cfg.n_features, n_img=P, n_pairs=P, channels=5, matchings=1) if c5 else
                  frame_bytes(width, height, cfg.n_features, n_img=2 * P, n_pairs=P))   # per rig frame
    front = ("rectify_pyramid", "detect", "select", "describe")
    dom = max(per_kernel_us, key=per_kernel_us.get)
    # front kernels (and, RGB-D, the whole per-camera back end) cover S of C cameras for B frames;
    # the other back kernels all cameras for B / N frames
    share = (S / C) * B if (dom in front or (c5 and dom != "rig")) else B / world
    dom_bytes = unit_bytes * share
    achieved = dom_bytes / (per_kernel_us[dom] * 1e-6) / 1e9
    alltoall = args.exchange == "alltoall" or c5 or args.driver == "library"
    if c5:
        xbytes = {"pair_blocks": (world - 1) * plan.frames_per_rank * S * pb, "pose_records": plan.frames_per_rank * pr,
                  "pair_block_bytes": pb, "pose_record_bytes": pr}
        xbytes["largest_to_one_peer"] = plan.frames_per_rank * S * pb
    elif args.driver == "library" and args.pair_split:
        # rank 0 (pair 0, first half) sends its camera of the partner's half + the frame before it
        # to the partner, and its pair's blocks of each rig range of the same half to that range's
        # owner (world / 2 - 1 ranks)
        half = B - B // 2
        xbytes = {
            "raw_images": (half + 1) * width * height,
            "stream_blocks": (half + 1) * sb,
            "pair_blocks": (world // 2 - 1) * plan.frames_per_rank * pb if P > 1 else 0,
            "pose_records": plan.frames_per_rank * pr,
            "stream_block_bytes": sb,
            "pair_block_bytes": pb,
            "pose_record_bytes": pr,
        }
        xbytes["largest_to_one_peer"] = (half + 1) * (width * height + sb)   # the partner link
    else:
        xbytes = {  # what one rank sends per step
            "raw_images": ((world - 1) * plan.recv_frames if alltoall else (B + 1)) * S * width * height,
            "stream_blocks": ((world - 1) * plan.recv_frames if alltoall else (B + 1)) * S * sb,
            "pose_records": plan.frames_per_rank * pr,
            "stream_block_bytes": sb,
            "pose_record_bytes": pr,
        }
        if alltoall:
            xbytes["largest_to_one_peer"] = plan.recv_frames * S * (width * height + sb)
    xbytes["total_sent"] = sum(v for k_, v in xbytes.items() if not k_.endswith("_bytes") and k_ != "largest_to_one_peer")
    if args.driver == "library":
        if rehearse:
            grp.close()
        for h in hs:
            h.close()
    else:
        rig.close()
    frames_total = args.steps * B        # rig frames
    value = frames_total / elapsed * (1 if (c3 or c5) else P)
    out = {
        "metric": METRIC_C3 if c3 else METRIC_C5 if c5 else METRIC,
        "value": value,
        "unit": "frames/s",
        "n_gpus": 1 if rehearse else world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong" if (c3 or c5) else "weak",
        "vs_baseline": None,
        "dtype": "u8+f64",
        "data": f"synthetic: seeded room renderer, {args.unique} distinct {width}x{height} frames of each rank's camera "
                f"streams (bracket rig, one shared room) replayed as a triangle wave, resident in HBM before timing",
        "config": {
            "workload": ("C5: 4-camera RGB-D rig (brackets.urdf joints), 1280x720 BGR + aligned u16 depth per camera, "
                         "2000 FAST/rBRIEF keypoints, temporal Hamming + depth-lookup 3D points + P3P-RANSAC(128)+GN "
                         "per camera, rig pose by generalised PnP over all cameras" if c5 else
                         ("C3: 4x OAK stereo rig (8 streams, brackets.urdf joints, sources of run_slam.py:45-50)"
                          if c3 else f"C2 streams over {world} GPUs: {P} stereo source(s) of the bracket rig "
                                     f"({C} streams), one camera stream per GPU")
                         + ", 640x400, 2000 FAST/rBRIEF keypoints per image, per-pair stereo+temporal Hamming + "
                           "P3P-RANSAC(128)+GN" + (", rig pose by generalised PnP over all pairs" if P > 1 else "")),
            "frames_per_step": B,
            "streams": C,
            "stereo_pairs": P,
            "n_features": cfg.n_features,
            "parallelism": (f"{S} RGB-D camera(s) per GPU x{world}: each GPU tracks its cameras over the batch, "
                            f"RCCL all-to-all of pair blocks (pose + correspondences), rig pose on each GPU's "
                            f"{plan.frames_per_rank}-frame range, RCCL all-gather of pose records" if c5 else
                            f"1 camera stream per GPU x{world}, pair split: front end per stream, RCCL send/recv of "
                            f"raw images + keypoint/descriptor stream blocks to the pair partner only, the pair's back "
                            f"end on each GPU's half of the batch, pair blocks to the rig-range owners of the same "
                            f"half, rig pose on each GPU's {plan.frames_per_rank}-frame range, RCCL all-gather of "
                            f"pose records" if (args.driver == "library" and args.pair_split) else
                            f"{S} camera stream(s) per GPU x{world}: front end per stream, RCCL "
                            f"{'all-to-all' if alltoall else 'all-gather'} of raw images + keypoint/descriptor "
                            f"stream blocks, per-pair back end + rig pose on each GPU's {plan.frames_per_rank}-frame "
                            f"range, RCCL all-gather of pose records"),
        },
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                     "algorithmic_bytes_per_launch": dom_bytes, "algorithmic_bytes_per_rig_frame": unit_bytes,
                     "avg_launch_us": per_kernel_us[dom], "rank": rank},
        "per_kernel_us_per_batch": per_kernel_us,
        "exchange_bytes_per_step": xbytes,
        # exchange_exposed: front end packed -> both exchanges landed on the back stream (what the
        # overlap does not hide); pose_gather: the pose-record all-gather on the back stream
        "exchange_us": exchange_us,
        "backend": (f"library driver, copy transport: {world} ranks on one GPU (rehearsal of the exchange, not a "
                    f"scaling value)" if rehearse else "library driver (tslam_comm_init + tslam_submit_sharded), RCCL"
                    if args.driver == "library" else f"torch.distributed {args.dist_backend} (DistShardedRig test double)"),
        "ranks": world,
        "tracking_ok_fraction_last_batch": ok,
        "rig_ok_fraction_last_batch": rig_ok,
        "render_s": t_render,
    }
    if c3:
        out["stereo_pair_frames_per_s"] = value * P
    elif c5:
        out["camera_frames_per_s"] = value * P
    else:
        out["rig_frames_per_s"] = frames_total / elapsed
    return out


def free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return int(s.getsockname()[1])


def launch_command(n: int, argv: list[str], port: int, script: str | os.PathLike | None = None) -> list[str]:
    """The torch.distributed.run command of an N-rank bench (one process per GPU, rendezvous on
    127.0.0.1; each rank reads RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* from its env)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", f"--master-port={port}", str(script or ROOT / "bench.py"), *argv]


def self_launch(n: int, argv: list[str], timeout_s: float, script: str | os.PathLike | None = None) -> int:
    """Run the N ranks as a child process group and return its exit code (124 when it runs past
    ``timeout_s``: the whole group is killed, so a rank stuck in RCCL init cannot hang the bench).
    Rank 0's JSON line reaches stdout through the inherited descriptors."""
    import signal

    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR",
                                                            "MASTER_PORT", "LOCAL_WORLD_SIZE")}
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # dmabuf IPC for RCCL on this host driver
    cmd = launch_command(n, argv, free_port(), script)
    proc = subprocess.Popen(cmd, env=env, start_new_session=True)
    try:
        return proc.wait(timeout=timeout_s)
    except subprocess.TimeoutExpired:
        print(f"bench: {n}-rank run exceeded {timeout_s:.0f} s; killing it", file=sys.stderr, flush=True)
        os.killpg(proc.pid, signal.SIGKILL)
        proc.wait()
        return 124


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", choices=["c2", "c3", "c4", "c5"], default="c2",
                    help="BASELINE.json configs[1] (c2), configs[2] (c3), configs[3] (c4) or configs[4] (c5)")
    ap.add_argument("--batch", type=int, default=0, help="frames per step (0 = C2_BATCH for c2, 256 for c3, 50 for c4, 128 for c5)")
    ap.add_argument("--unique", type=int, default=0, help="distinct rendered frames, triangle-wave replay (0 = C2_UNIQUE for c2, 48 for c3, 24 for c4 / c5)")
    ap.add_argument("--cpu-budget", type=float, default=12.0, help="seconds of oracle CPU baseline (0 = skip)")
    ap.add_argument("--cpu-procs", type=int, default=0, help="oracle processes for the CPU baseline (0 = usable CPUs)")
    ap.add_argument("--latency-frames", type=int, default=20, help="B=1 submissions timed for latency_b1_ms")
    ap.add_argument("--boundary-frames", type=int, default=1024,
                    help="c2: frames timed through HipSlamEngine.process_frames (0 = skip)")
    ap.add_argument("--default-frames", type=int, default=1024,
                    help="c2: frames timed through the reference's default construction (batch 1, loop closure + "
                         "IMU on) for C2 and (half as many) the C3 rig, in boundary.default_config (0 = skip)")
    ap.add_argument("--out", type=str, default="", help="also write the JSON line to this file")
    ap.add_argument("--outliers", type=int, default=35,
                    help="c2/c3: also time --outlier-steps pipelined steps with this %% of the refined temporal "
                         "positions made outliers before the pose kernels (pose_with_outliers; 0 = skip)")
    ap.add_argument("--outlier-steps", type=int, default=5)
    ap.add_argument("--dist-backend", type=str, default="nccl", help="nccl (RCCL) or gloo (rehearsal, host copy)")
    ap.add_argument("--exchange", choices=["alltoall", "allgather"], default="alltoall",
                    help="--driver torch: all-to-all of the frames each rank solves, or all-gather of everything")
    ap.add_argument("--driver", choices=["library", "torch"], default="library",
                    help="sharded rig: the library's own driver (shipped; RCCL from tslam_comm_init) or the "
                         "torch.distributed test double (thor_slam_amd/shard.py)")
    ap.add_argument("--transport", choices=["rccl", "copy"], default="rccl",
                    help="copy: all --gpus ranks in this process on one GPU with device copies (tslam_group_create; "
                         "a rehearsal of the library driver's exchange on a one-GPU box)")
    ap.add_argument("--pair-split", type=int, default=0,
                    help="sharded stereo rig, one camera per GPU: TSLAM_SHARD_PAIRS (each rank solves its camera's "
                         "pair over half the batch; images go to the partner only, pair blocks to the rig ranges)")
    ap.add_argument("--pipeline", type=int, default=1,
                    help="1: front and back kernels on two streams (batch s+1's front overlaps batch s's back)")
    ap.add_argument("--front-cu-reserve", type=int, default=-1,
                    help="C4: keep the front / back kernels off the last N CUs (left to the BA chain); "
                         "-1 = the C4 default, 96 (round 5 sweep after the BA preparation changes: 32 / 64 / 96 / "
                         "128 CUs -> 16.9k / 17.55k / 17.66k / 17.48k frames/s; round 4: 0 / 32 / 48 / 64 / 80 / 96 / "
                         "128 -> 15.1k / 15.6k / 15.7k / 16.2k / 15.9k / 16.2k / 16.0k)")
    ap.add_argument("--back-cu", type=int, default=0,
                    help="experiment (c2/c3): the back kernels on a stream restricted to N CUs spread over the chip")
    ap.add_argument("--split-cu", type=int, default=0,
                    help="experiment (c2/c3, with --back-cu N): the front kernels on the other CUs, disjoint from the back's")
    ap.add_argument("--ba-priority", type=int, default=0, help="C4: the BA stream at high priority")
    ap.add_argument("--ba-defer", type=int, default=1,
                    help="C4: enqueue each batch's BA launches at the next batch's first back stage (tslam_ba_defer)")
    ap.add_argument("--ba-cus", type=int, default=0,
                    help="C4 experiment: the BA stream CU-masked to the last N CUs (with --front-cu-reserve N "
                         "the front / back kernels keep off them)")
    ap.add_argument("--front-priority", type=int, default=1,
                    help="1: run the front kernels on a high-priority stream (pipelined mode)")
    ap.add_argument("--tsdf", type=int, default=0,
                    help="c5: also integrate every batch's depth into a TSDF volume with the device poses "
                         "(nvblox-shaped dense map, SURVEY.md §8f item 4); reported under dense_map")
    ap.add_argument("--kernel-events", type=str, default="detect,local_ba,tsdf",
                    help="kernels timed with HIP events inside the timed steps: 'all' or a comma list "
                         "(default: the roofline kernel detect, C4 BA stage, C5 TSDF)")
    ap.add_argument("--pmc", type=str, default=str(ROOT / "profiles" / "pmc_latest.json"),
                    help="PMC summary (tools/pmc_summary.py) used for roofline.traffic when its batch matches")
    ap.add_argument("--launch-timeout", type=float, default=1500.0,
                    help="--gpus N > 1 without WORLD_SIZE: seconds before the self-launched ranks are killed")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1 and args.transport != "copy":
        # N ranks requested from a plain `python bench.py --gpus N`: launch them (before this
        # process touches the GPU) and report rank 0's line
        sys.exit(self_launch(args.gpus, sys.argv[1:], args.launch_timeout))

    import torch
    import torch.distributed as dist

    rehearse = args.transport == "copy"
    world = args.gpus if rehearse else int(os.environ.get("WORLD_SIZE", "1"))
    rank = 0 if rehearse else int(os.environ.get("RANK", "0"))
    local = 0 if rehearse else int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if world > 1 and not rehearse and args.dist_backend == "nccl" and world > torch.cuda.device_count():
        raise SystemExit(f"--gpus {world} over RCCL needs one GPU per rank ({torch.cuda.device_count()} visible); "
                         "use --transport copy to rehearse the library driver's ranks on one GPU "
                         "(or --dist-backend gloo --driver torch for the torch.distributed test double)")
    if args.config == "c4" and world > 1:
        raise SystemExit("--config c4 is a single-GPU configuration")
    dev_index = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev_index)
    if world > 1 and not rehearse:
        import datetime

        # a collective (or the communicator's eager init) that does not complete in this time
        # aborts the rank with an error instead of hanging the job
        tmo = datetime.timedelta(seconds=300)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_index), timeout=tmo)
        else:
            dist.init_process_group(args.dist_backend, timeout=tmo)
    if world > 1 and not rehearse and args.driver == "library" and args.dist_backend != "nccl":
        raise SystemExit("the library driver exchanges over RCCL: --dist-backend nccl (or --transport copy)")
    sharded = world > 1 and args.config in ("c2", "c3", "c5")
    out = run_sharded(args, world, rank, dev_index) if sharded else run_single(args, world, rank, dev_index)
    if world > 1 and not rehearse:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        line = json.dumps(out)
        print(line, flush=True)
        if args.out:
            Path(args.out).write_text(line + "\n")


if __name__ == "__main__":
    main()
