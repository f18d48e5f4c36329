"""Throughput bench: synced stereo frames/sec (detect + match + pose) @ 640x400 on MI355X.

python bench.py --gpus N --steps K --warmup W   (N > 1 under torch.distributed.run, one rank/GPU)
python bench.py --config c4                     (BASELINE.json configs[3]: 1280x800, K=4000, + local BA)
python bench.py --config c5 [--gpus 4]          (BASELINE.json configs[4]: RGB-D 1280x720, one camera per GPU)

* workload (BASELINE.json configs[1], C2): one stereo pair 640x400 per GPU, K=2000 ORB-style
  keypoints per image, synthetic room sequence (seed = rank); a *step* = one batch of
  ``--batch`` synchronised stereo frames pushed through the whole hot path
  (rectify -> pyramid -> FAST/NMS/top-K -> orientation + rBRIEF -> stereo + temporal Hamming
  match -> sub-pixel refinement -> P3P-RANSAC -> Gauss-Newton -> pose chaining).
* inputs are rendered on the host before timing and are resident in HBM (a triangle-wave
  replay of ``--unique`` rendered frames, so consecutive frames stay consecutive in time).
* N > 1: weak scaling, one stereo source per rank; each step also all-gathers the packed
  keypoint + descriptor block of every rank over RCCL (the exchange step of SURVEY.md §8e).
* timing: barrier + synchronize on both sides of exactly K steps; MAX over ranks.
* roofline: per-kernel HIP-event timing of one batch run kernel by kernel on the same stream,
  for the dominant kernel: algorithmic bytes / average duration vs 8 TB/s.
* cpu_baseline (rank 0, N=1 context): the NumPy oracle on a bounded sample of the same frames.
* --config c4: the same step plus the A8 stage (every 5th frame a keyframe of a 10-keyframe
  window, 5 Gauss-Newton iterations per keyframe); the roofline is then that of the dominant
  kernel of the step, the FP64-MFMA Schur product when it dominates (HIP events around its launches).
* --config c5: RGB-D frames (BGR u8 + aligned u16 mm depth, 1280x720) of one camera per GPU; the
  colour image is converted on the device and depth replaces the stereo matching.
"""

from __future__ import annotations

import argparse
import json
import os
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
METRIC_C4 = "synced stereo frames/sec (detect+match+pose+10-keyframe local BA) @1280×800, 1 GPU"
METRIC_C5 = "RGB-D frames/sec (BGR+depth, detect+match+pose) @1280×720, one camera per GPU, 1/2/4 GPU"
HBM_PEAK_GBS = 8000.0
# VALU issue: 256 CUs x 4 SIMD-32, a wave64 instruction every 2 cycles per SIMD at 2.4 GHz
VALU_PEAK_WINST = 256 * 4 * 2.4e9 / 2
FP64_MFMA_PEAK_TFS = 78.6   # MI355X FP64 matrix peak (AMD spec; the microarch guide lists no FP64 row)
# bench kernel label -> device symbol (rocprofv3 / PMC summaries); "pose" is k_corr+k_ransac+k_refine
KERNEL_SYMBOL = {"rectify_pyramid": "k_rectify_pyramid", "detect": "k_detect", "select": "k_select",
                 "describe": "k_describe", "match": "k_match", "match_refine": "k_refine_temporal",
                 "pose": "k_ransac", "chain": "k_chain"}


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


def triangle_indices(total: int, unique: int) -> np.ndarray:
    period = 2 * (unique - 1)
    k = np.arange(total) % period
    return np.where(k < unique, k, period - k)


def frame_bytes(W: int, H: int, K: int, n_img: int = 2, n_pairs: int = 1, channels: int = 1, matchings: int = 2) -> int:
    """SURVEY.md §8d compulsory bytes per stereo frame: read the images, write keypoints (12 B) and
    descriptors (32 B), write the match records (8 B per keypoint, for the stereo and the temporal
    matching of each pair).  C2: 2 * (256,000 + 88,000) + 2 * 16,000 = 720,000 B.  RGB-D (C5): one
    image of 5 bytes per pixel (BGR + u16 depth), temporal matching only."""
    return n_img * (W * H * channels + K * (12 + 32)) + matchings * n_pairs * K * 8


def kernel_bytes(name: str, B: int, h, cfg, maps_identity: bool) -> float:
    """Algorithmic (compulsory) HBM bytes of one launch of a kernel over B stereo frames."""
    W, H, K = h.width, h.height, cfg.n_features
    imgs = 2 * B
    pyr = sum(w * hh for w, hh in h.level_wh)
    if name == "rectify_pyramid":
        maps = 0 if maps_identity else 2 * W * H * 8
        return imgs * (W * H + pyr) + maps
    if name == "detect":
        return imgs * (pyr + pyr)          # read the levels, write the smoothed levels
    if name == "select":
        return imgs * K * 8                # write keypoints (candidate reads are data-dependent)
    if name == "describe":
        return imgs * K * (8 + 32)         # read keypoints, write descriptors
    if name == "match":
        return B * 2 * (2 * K * 32 + K * 8)  # two matchings: read query+train descriptors, write best/second
    if name == "match_refine":
        return B * 2 * K * (8 + 16)
    if name == "pose":
        return B * K * (4 + 16 + 8 * 8)
    if name == "chain":
        return B * 68 * 8
    return 0.0


def _oracle_worker(args):
    """One CPU process: the NumPy oracle tracking its contiguous frame chunk (replayed) for budget_s."""
    frames, rect_d, cfg_d, budget_s = args
    if cfg_d.get("rgbd"):
        return _oracle_worker_rgbd(args)
    from oracle import numpy_slam as O
    from thor_slam_amd.params import HipSlamConfig

    cfg = HipSlamConfig(**cfg_d)
    trk = O.OracleTracker(cfg, rect_d)
    bat = None
    if cfg.ba_window > 0:
        from oracle.numpy_ba import BAParams, BATracker

        bat = BATracker(cfg.n_features, (rect_d["fx"], rect_d["fy"], rect_d["cx"], rect_d["cy"],
                                         rect_d["fx"] * rect_d["baseline"]),
                        BAParams(cfg.ba_window, cfg.ba_kf_interval, cfg.ba_iters, cfg.ba_lambda, cfg.ba_outlier_px))
    n = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < budget_s:
        i = n % len(frames)
        res = trk.step(frames[i, 0], frames[i, 1])
        if bat is not None:
            bat.step(res)
        n += 1
    return n, time.perf_counter() - t0


def _oracle_worker_rgbd(args):
    frames, rect_d, cfg_d, budget_s = args   # frames: (n, H, W, 3) BGR and (n, H, W) depth
    from oracle import numpy_slam as O
    from thor_slam_amd.params import HipSlamConfig

    bgr, depth = frames
    trk = O.OracleTracker(HipSlamConfig(**cfg_d), rect_d)
    n = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < budget_s:
        i = n % len(bgr)
        trk.step_rgbd(bgr[i], depth[i])
        n += 1
    return n, time.perf_counter() - t0


def cpu_baseline_rgbd(bgr: np.ndarray, depth: np.ndarray, rect, cfg, budget_s: float, procs: int) -> dict:
    import dataclasses

    rect_d = dict(fx=rect.fx, fy=rect.fy, cx=rect.cx, cy=rect.cy, baseline=rect.baseline,
                  map_l=rect.map_left, map_r=rect.map_right)
    cfg_d = dataclasses.asdict(cfg)
    parts = [(b, d) for b, d in zip(np.array_split(bgr, procs), np.array_split(depth, procs)) if len(b)]
    with ProcessPoolExecutor(max_workers=len(parts)) as ex:
        results = list(ex.map(_oracle_worker, [(pt, rect_d, cfg_d, budget_s) for pt in parts]))
    n = sum(r[0] for r in results)
    wall = max(r[1] for r in results)
    return {"value": n / wall, "unit": "frames/s", "cores": len(parts), "kind": "port",
            "sample": f"{n} synthetic {bgr.shape[2]}x{bgr.shape[1]} RGB-D frames (seed 0, {len(bgr)} distinct, replayed "
                      f"per process), NumPy oracle step_rgbd, {len(parts)} process(es) x {budget_s:.0f} s"}


def cpu_baseline(frames: np.ndarray, rect, cfg, budget_s: float, procs: int) -> dict:
    """The NumPy oracle on the host cores: `procs` processes, each tracking a contiguous chunk of the
    same frames (relative-pose work is independent per frame pair)."""
    import dataclasses

    rect_d = dict(fx=rect.fx, fy=rect.fy, cx=rect.cx, cy=rect.cy, baseline=rect.baseline,
                  map_l=rect.map_left, map_r=rect.map_right)
    cfg_d = dataclasses.asdict(cfg)
    chunks = [c for c in np.array_split(frames, procs) if len(c)]
    if len(chunks) == 1:
        results = [_oracle_worker((chunks[0], rect_d, cfg_d, budget_s))]
    else:
        with ProcessPoolExecutor(max_workers=len(chunks)) as ex:
            results = list(ex.map(_oracle_worker, [(c, rect_d, cfg_d, budget_s) for c in chunks]))
    n = sum(r[0] for r in results)
    wall = max(r[1] for r in results)
    return {"value": n / wall, "unit": "frames/s", "cores": len(chunks), "kind": "port",
            "sample": f"{n} synthetic {frames.shape[3]}x{frames.shape[2]} stereo frames (seed 0, {len(frames)} distinct, "
                      f"replayed per process), NumPy oracle{' + local BA' if cfg.ba_window else ''}, "
                      f"{len(chunks)} process(es) x {budget_s:.0f} s"}


# the synthetic room (8 x 8 x 3 m, FLU) in the tracking world (rect-left camera of frame 0, RDF):
# x in [-6.9, 1.1], y in [-1.5, 1.5], z in [-4, 4] m; the volume adds 0.3-0.5 m around it
TSDF_ORIGIN = (-7.2, -1.8, -4.4)
TSDF_DIMS = (176, 72, 176)


def tsdf_report(h, us: float, B: int, width: int, height: int) -> dict:
    """k_tsdf_integrate of one batch: voxel (tsdf, weight) read-modify-write once per launch
    (8 + 8 B per observed voxel) + the batch's depth images read once; the voxel-frame updates
    (the per-voxel projection work) beside it."""
    t, w = h.tsdf_read()
    nv = int(np.prod(TSDF_DIMS))
    observed = int((w > 0).sum())
    alg = nv * 16 + B * width * height * 2
    return {"kernel": "k_tsdf_integrate", "volume_voxels": nv, "voxel_size_m": 0.05, "truncation_voxels": 4,
            "frames_per_launch": B, "avg_launch_us": us, "observed_voxels": observed,
            "voxel_frame_updates_per_s": nv * B / (us * 1e-6),
            "roofline": {"bound": "hbm", "achieved": alg / (us * 1e-6) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": alg / (us * 1e-6) / 1e9 / HBM_PEAK_GBS, "algorithmic_bytes_per_launch": alg}}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", choices=["c2", "c4", "c5"], default="c2",
                    help="BASELINE.json configs[1] (c2), configs[3] (c4) or configs[4] (c5)")
    ap.add_argument("--batch", type=int, default=0, help="frames per step (0 = 256 for c2, 50 for c4, 128 for c5)")
    ap.add_argument("--unique", type=int, default=0, help="distinct rendered frames, triangle-wave replay (0 = 48 / 24)")
    ap.add_argument("--cpu-budget", type=float, default=12.0, help="seconds of oracle CPU baseline (0 = skip)")
    ap.add_argument("--cpu-procs", type=int, default=8, help="oracle processes for the CPU baseline")
    ap.add_argument("--latency-frames", type=int, default=20, help="B=1 submissions timed for latency_b1_ms")
    ap.add_argument("--out", type=str, default="", help="also write the JSON line to this file")
    ap.add_argument("--dist-backend", type=str, default="nccl", help="nccl (RCCL) or gloo (rehearsal, host copy)")
    ap.add_argument("--pipeline", type=int, default=1,
                    help="1: front and back kernels on two streams (batch s+1's front overlaps batch s's back)")
    ap.add_argument("--front-priority", type=int, default=1,
                    help="1: run the front kernels on a high-priority stream (pipelined mode)")
    ap.add_argument("--tsdf", type=int, default=0,
                    help="c5: also integrate every batch's depth into a TSDF volume with the device poses "
                         "(nvblox-shaped dense map, SURVEY.md §8f item 4); reported under dense_map")
    ap.add_argument("--pmc", type=str, default=str(ROOT / "profiles" / "pmc_latest.json"),
                    help="PMC summary (tools/pmc_summary.py) used for roofline.traffic when its batch matches")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    from thor_slam_amd._lib import KERNELS, Handle
    from thor_slam_amd.calib import extract_cameras, stereo_pairs, stereo_rectify
    from thor_slam_amd.dist import BlockLayout, FeatureExchange
    from thor_slam_amd.camera.rig import CameraRig
    from thor_slam_amd.params import HipSlamConfig
    from thor_slam_amd.rgbd import pack_rgbd
    from thor_slam_amd.synthetic import SyntheticStereoSource

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    dev_index = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev_index)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_index))
        else:
            dist.init_process_group(args.dist_backend)

    c4, c5 = args.config == "c4", args.config == "c5"
    if c4 and world > 1:
        raise SystemExit("--config c4 is a single-GPU configuration")
    width, height = (1280, 800) if c4 else (1280, 720) if c5 else (640, 400)
    cfg = (HipSlamConfig(n_features=4000, ba_window=10, ba_kf_interval=5, ba_iters=5) if c4 else
           HipSlamConfig(rgbd=True) if c5 else HipSlamConfig())
    B = args.batch or (50 if c4 else 128 if c5 else 256)
    args.unique = args.unique or (24 if (c4 or c5) else 48)
    workers = max(1, min(16, (os.cpu_count() or 2) // max(1, world), args.unique))
    t_r = time.perf_counter()
    if c5:
        from thor_slam_amd.calib import rgbd_pairs, rgbd_undistort
        from thor_slam_amd.synthetic import SyntheticRGBDSource

        src = SyntheticRGBDSource(seed=rank, n_frames=args.unique, width=width, height=height)
        cams = extract_cameras(CameraRig([src]).calibration, 2)
        (ci, _), = rgbd_pairs(cams)
        rect = rgbd_undistort(cams[ci])
        rgbd_frames = [src.render_rgbd(i) for i in range(args.unique)]
        uniq = np.stack([pack_rgbd(b, d) for b, d in rgbd_frames])[:, None, :]   # [n][1][5HW]
    else:
        src = SyntheticStereoSource(seed=rank, n_frames=args.unique, width=width, height=height)
        cams = extract_cameras(CameraRig([src]).calibration, 2)
        (li, ri), = stereo_pairs(cams)
        rect = stereo_rectify(cams[li], cams[ri])
        uniq = render_frames(rank, args.unique, workers, width, height)
    t_render = time.perf_counter() - t_r

    total = (args.warmup + args.steps) * B
    idx = torch.from_numpy(triangle_indices(total, args.unique)).cuda()
    seq = torch.from_numpy(uniq).cuda().index_select(0, idx).contiguous()  # [total, 2, H, W] (c5: [total, 1, 5HW]) in HBM
    h = Handle([rect], cfg, max_batch=B, device=dev_index)
    # the front stream (rectify .. describe) is the critical path of the pipelined step: with
    # --front-priority 1 it is a high-priority stream, so the back kernels fill the gaps around it
    stream = (torch.cuda.Stream(priority=-1) if args.front_priority and args.pipeline else torch.cuda.current_stream())
    torch.cuda.set_stream(stream)
    sp = stream.cuda_stream
    layout = BlockLayout(n_frames=B, n_cams=1 if c5 else 2, K=cfg.n_features, L=cfg.n_levels)
    on_device = args.dist_backend == "nccl"
    # two exchange buffers: batch s packs into buffer s % 2 and all-gathers it asynchronously over
    # RCCL while batch s + 1 computes (the buffer is reused only after its gather has completed)
    exchanges = [FeatureExchange(layout, "cuda" if on_device else "cpu", world) for _ in range(2)] if world > 1 else []
    pending = {"work": None, "buf": 0, "batch": -1}   # the in-flight all-gather (one at a time)
    staging = torch.empty((layout.rank_bytes,), dtype=torch.uint8, device="cuda") if world > 1 and not on_device else None
    recv_dev = None
    if world > 1:
        # the rig-level solve after the gather: every rank fuses all ranks' body
        # motions on its device; the rig extrinsics of every rank's pair are exchanged once
        bt = torch.from_numpy(np.ascontiguousarray(cams[0].extrinsics.to_4x4_matrix() @ rect.left_optical_T_rect()))
        if on_device:
            every = torch.empty((world, 4, 4), dtype=torch.float64, device="cuda")
            dist.all_gather_into_tensor(every, bt.cuda())
            every = every.cpu()
        else:
            parts = [torch.empty((4, 4), dtype=torch.float64) for _ in range(world)]
            dist.all_gather(parts, bt)
            every = torch.stack(parts)
            recv_dev = torch.empty((world * layout.rank_bytes,), dtype=torch.uint8, device="cuda")
        h.set_rig_ranks(list(every.numpy()))
    names = list(KERNELS) + (["local_ba"] if c4 else []) + (["tsdf"] if c5 and args.tsdf else [])
    if c5 and args.tsdf:
        h.tsdf_init(TSDF_ORIGIN, TSDF_DIMS, 0.05, 4.0, 10.0, 100.0)
    BACK = {"match", "match_refine", "pose", "chain"}
    # two streams: the front kernels (rectify .. describe) of batch s + 1 overlap the back kernels
    # (match .. chain) of batch s; the library orders batch s's back after its front and batch s's
    # front after the back of batch s - 2 (ring slots); the exchange and fusion follow the back.
    bstream = torch.cuda.Stream() if args.pipeline else stream
    bsp = bstream.cuda_stream
    back_done = [torch.cuda.Event(), torch.cuda.Event()]
    back_issued = [False, False]
    # C4: local BA runs on a third stream, overlapping the next batches
    ba_stream = torch.cuda.Stream() if c4 else None
    ba_done = [torch.cuda.Event(), torch.cuda.Event()] if c4 else None
    ba_issued = [False, False]

    def finish_exchange() -> None:
        """Make the back stream wait for the in-flight gather (the host does not block) and run the
        rig fusion of that batch on the device."""
        if pending["work"] is not None:
            with torch.cuda.stream(bstream):
                pending["work"].wait()
            h.rig_fuse(exchanges[pending["buf"]].recv.data_ptr(), world, pending["batch"] * B, B, bsp)
            pending["work"] = None

    def step(s: int, evs=None) -> None:
        # one batch = every kernel of the hot path; in the timed steps each kernel is bracketed by
        # a pair of HIP events on the stream it runs on (the per-kernel durations below)
        h.begin_batch(seq[s * B].data_ptr(), B)
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
                h.run_stage("ba", ba_stream.cuda_stream)
                ba_done[s % 2].record(ba_stream)
                ba_issued[s % 2] = True
                if evs is not None:
                    evs[i][1].record(ba_stream)
                continue
            st = bstream if k in BACK else stream
            if k in BACK and first_back and bstream is not stream:
                bstream.wait_stream(stream)
                first_back = False
            if evs is not None:
                evs[i][0].record(st)
            h.run_kernel(k, st.cuda_stream)
            if evs is not None:
                evs[i][1].record(st)
        if bstream is not stream:
            back_done[s % 2].record(bstream)
            back_issued[s % 2] = True
        h.end_batch()
        if "tsdf" in names:   # the batch's depth into the volume, with its device-resident poses
            i = names.index("tsdf")
            if evs is not None:
                evs[i][0].record(bstream)
            h.tsdf_integrate(seq[s * B].data_ptr() + 3 * width * height, 5 * width * height, B,
                             first_frame=s * B, stream=bsp)
            if evs is not None:
                evs[i][1].record(bstream)
        if exchanges:  # the exchange step: every rank's keypoints/descriptors/poses to all ranks
            k = s % 2
            ex = exchanges[k]
            if on_device:
                # batch s-1's gather ran while batch s computed: fuse it, then ship batch s
                finish_exchange()
                h.pack_features(ex.send.data_ptr(), bsp)
                with torch.cuda.stream(bstream):
                    pending.update(work=ex.all_gather(async_op=True), buf=k, batch=s)
            else:   # gloo rehearsal: host gather, then the same device fusion
                h.pack_features(staging.data_ptr(), bsp)
                bstream.synchronize()
                ex.send.copy_(staging.cpu())
                ex.all_gather()
                with torch.cuda.stream(bstream):
                    recv_dev.copy_(ex.recv)
                h.rig_fuse(recv_dev.data_ptr(), world, s * B, B, bsp)

    def drain() -> None:
        finish_exchange()

    events = [[(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in names]
              for _ in range(args.steps)]
    for s in range(args.warmup):
        step(s)
    drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    if c4:   # arm the Schur-kernel events (launches per step: keyframes x iterations)
        h.ba_profile(max_launches=args.steps * (B // cfg.ba_kf_interval + 1) * cfg.ba_iters)
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(args.warmup + k, events[k])
    drain()
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
    ok_frac = float(np.mean(res["stats"][:, 0, 0] == 0))
    rig_ok = None
    if world > 1:
        rig_ok = float(np.mean(h.read_rig_poses(B)["stats"][:, 0] == 0))

    # ---- the same kernels run alone (after the timed region, one stream, 3 batches): under the
    # two-stream pipeline a kernel shares the GPU with the other stream's kernels, so its timed
    # duration above includes that sharing; these isolated durations are the kernel's own speed
    iso_us = {k: 0.0 for k in KERNELS}
    n_iso = 3
    torch.cuda.synchronize()
    for r in range(n_iso):
        s_iso = r % (args.warmup + args.steps)   # replayed input: only the durations are used
        h.begin_batch(seq[s_iso * B].data_ptr(), B)
        pairs = []
        for k in KERNELS:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            h.run_kernel(k, sp)
            e1.record(stream)
            pairs.append((k, e0, e1))
        h.end_batch()
        torch.cuda.synchronize()
        for k, e0, e1 in pairs:
            iso_us[k] += e0.elapsed_time(e1) * 1e3 / n_iso

    # ---- per-kernel durations of the timed launches (HIP events on the launch stream) ----------
    per_kernel_us = {k: 0.0 for k in names}
    for evs in events:
        for i, k in enumerate(names):
            per_kernel_us[k] += evs[i][0].elapsed_time(evs[i][1]) * 1e3 / args.steps  # us
    unit_bytes = (frame_bytes(rect.width, rect.height, cfg.n_features, n_img=1, channels=5, matchings=1) if c5 else
                  frame_bytes(rect.width, rect.height, cfg.n_features))
    dom_bytes = unit_bytes * B          # §8d per-frame bytes x the frames one launch processes
    schur = h.ba_profile(0) if c4 else None
    front = {k: v for k, v in per_kernel_us.items() if k not in ("local_ba", "tsdf")}
    dom = max(front, key=front.get)
    achieved = dom_bytes / (per_kernel_us[dom] * 1e-6) / 1e9
    mfma = None
    if schur and schur["launches"]:
        avg_us = schur["ms"] * 1e3 / schur["launches"]
        flops = schur["flops"] / schur["launches"]
        mfma = {"bound": "mfma", "kernel": "k_ba_schur", "achieved": flops / (avg_us * 1e-6) / 1e12,
                "peak": FP64_MFMA_PEAK_TFS, "unit": "TFLOP/s", "traffic": None, "dtype": "f64",
                "algorithmic_flops_per_launch": flops, "avg_launch_us": avg_us, "launches_timed": schur["launches"],
                "time_per_step_us": schur["ms"] * 1e3 / args.steps}
        mfma["frac"] = mfma["achieved"] / mfma["peak"]

    traffic = None
    valu = None
    pmc_path = Path(args.pmc)
    if pmc_path.exists():
        pmc = json.loads(pmc_path.read_text())
        kern = pmc.get("kernels", {}).get(KERNEL_SYMBOL.get(dom, ""), None)
        if kern is not None and pmc.get("batch_frames") == B and pmc.get("config", "c2") == args.config:
            traffic = kern["hbm_bytes_per_launch"]
            if kern.get("valu_insts_per_launch"):
                # the path is integer-VALU bound: wave64 VALU instructions per launch
                # (PMC SQ_INSTS_VALU) / the same event-timed duration, against the issue peak
                rate = kern["valu_insts_per_launch"] / (per_kernel_us[dom] * 1e-6)
                valu = {"bound": "valu", "achieved": rate / 1e12, "peak": VALU_PEAK_WINST / 1e12,
                        "unit": "T wave-instructions/s", "frac": rate / VALU_PEAK_WINST,
                        "insts_per_launch": kern["valu_insts_per_launch"]}

    # ---- B = 1 latency: one frame submitted and its pose read back -------------
    lat_ms = None
    if rank == 0 and args.latency_frames > 0:
        h1 = Handle([rect], cfg, max_batch=1, device=dev_index)
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
        "algorithmic_bytes_per_launch": dom_bytes,
        "algorithmic_bytes_per_frame": unit_bytes,
        "frames_per_launch": B,
        "avg_launch_us": per_kernel_us[dom],
        "kernel_own_bytes_per_launch": None if c5 else kernel_bytes(dom, B, h, cfg, rect.is_identity),
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
        workload = ("C5: one RGB-D camera per GPU, 1280x720 BGR u8 + aligned u16 mm depth, on-device gray conversion, "
                    "2000 FAST/rBRIEF keypoints, 4 levels, temporal brute-force Hamming, depth-lookup 3D points, "
                    "P3P-RANSAC(128)+GN pose")
    elif c4:
        workload = ("C4: 1x stereo pair 1280x800, 4000 FAST/rBRIEF keypoints per image, 4 levels, stereo+temporal "
                    "brute-force Hamming, P3P-RANSAC(128)+GN pose, 10-keyframe local BA (keyframe every 5 frames, "
                    "5 Gauss-Newton iterations, Schur complement on FP64 MFMA)")
    else:
        workload = ("C2: 1x stereo pair 640x400 per GPU, 2000 FAST/rBRIEF keypoints per image, 4 levels, "
                    "stereo+temporal brute-force Hamming, P3P-RANSAC(128)+GN pose")
    out = {
        "metric": METRIC_C4 if c4 else METRIC_C5 if c5 else METRIC,
        "value": frames_total / elapsed,
        "unit": "frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8" + ("+f64" if c4 else ""),
        "data": f"synthetic: seeded room renderer, {args.unique} distinct {width}x{height} "
                f"{'RGB-D' if c5 else 'stereo'} frames per rank replayed as a triangle wave, resident in HBM before timing",
        "config": {
            "workload": workload,
            "frames_per_step": B,
            "n_features": cfg.n_features,
            "parallelism": f"one {'RGB-D camera' if c5 else 'stereo source'} per GPU x{world}"
                           + (" + RCCL all-gather of keypoints/descriptors/poses + on-device rig fusion"
                              if world > 1 else ""),
        },
        "roofline": roofline,
        "latency_b1_ms": lat_ms,
        "per_kernel_us_per_batch": per_kernel_us,
        "per_kernel_us_isolated": iso_us,
        "tracking_ok_fraction_last_batch": ok_frac,
        "rig_fusion_ok_fraction_last_batch": rig_ok,
        "render_s": t_render,
    }
    if front_roofline is not None:
        out["front_end_roofline"] = front_roofline
    if "tsdf" in names:
        out["dense_map"] = tsdf_report(h, per_kernel_us["tsdf"], B, width, height)
    if rank == 0 and args.cpu_budget > 0:
        if c5:
            out["cpu_baseline"] = cpu_baseline_rgbd(np.stack([b for b, _ in rgbd_frames]), np.stack([d for _, d in rgbd_frames]),
                                                    rect, cfg, args.cpu_budget, args.cpu_procs)
        else:
            out["cpu_baseline"] = cpu_baseline(uniq, rect, cfg, args.cpu_budget, args.cpu_procs)
        out["cpu_baseline"]["host_cpus_visible"] = os.cpu_count()
    h.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        line = json.dumps(out)
        print(line, flush=True)
        if args.out:
            Path(args.out).write_text(line + "\n")


if __name__ == "__main__":
    main()
