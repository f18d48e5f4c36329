"""The sharded rig's per-rank work in a one-GPU rehearsal of the library driver (profiling aid).

    python tools/shard_probe.py [--world 8] [--batch 256] [--names 4] [--steps 4] [--one-gpu] [--pairs]

All `world` ranks of a tslam_group (copy transport) on this GPU with TSLAM_SHARD_SERIAL |
TSLAM_SHARD_PROFILE: every kernel and copy of every rank runs alone on one stream and is timed
with HIP events by the driver itself (tslam_shard_timing: rectify .. describe, stream-block pack,
import of the peers' raw images + stream blocks, match .. rig pose, the pose all-gather, the
chain).  Prints per rank the µs per step of each segment and its per-GPU compute (the segments
without the device copies standing in for RCCL, run one after another), then rank 0's pipelined
step alone on the GPU (TSLAM_SHARD_SOLO | TSLAM_SHARD_PIPELINE: front end of batch s+1 beside the
back end of batch s, exchanges skipped) — the N-GPU step when the exchange is hidden —
the bytes one rank sends per step, and (--one-gpu) the one-GPU step of the same rig and batch
through the pipelined single handle for the ratio.  --pairs runs the pair split (TSLAM_SHARD_PAIRS:
one camera per rank, the partner's images only, pair blocks to the rig ranges).
"""

from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for p in (ROOT, ROOT / "thor-slam_amd"):
    sys.path.insert(0, str(p))

EXCHANGE = ("exchange_wait", "pose_gather")   # device copies standing in for RCCL (and waits)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--names", type=int, default=4, help="stereo sources of the bracket rig (2 streams each)")
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--one-gpu", action="store_true", help="also time the one-GPU pipelined step (bench run_single)")
    ap.add_argument("--refine-block", type=int, default=0, help="tslam_params.refine_block (0 = the library's choice)")
    ap.add_argument("--pairs", action="store_true", help="TSLAM_SHARD_PAIRS (world = 2 x names)")
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    import torch

    from bench import RIG_SOURCES, render_rig_frames, rig_setup, triangle_indices
    from thor_slam_amd._lib import Handle, HandleGroup
    from thor_slam_amd.params import HipSlamConfig

    names = RIG_SOURCES[:args.names]
    _, cams, pairs, rects, E = rig_setup(names)
    C, B, W = 2 * len(rects), args.batch, args.world
    S = C // W
    cfg = HipSlamConfig()
    uniq = render_rig_frames(names, 24, 0, C, 8)
    seq = torch.from_numpy(uniq[triangle_indices((args.steps + 1) * B, 24)]).cuda()
    parts = [seq[:, r * S:(r + 1) * S].contiguous() for r in range(W)]
    hs = [Handle(rects, cfg, max_batch=B, refine_block=args.refine_block) for _ in range(W)]
    for h in hs:
        if len(rects) > 1:
            h.set_rig(E)
    grp = HandleGroup(hs, "copy")
    pairs = args.pairs
    hs[0].shard_options(serial=True, pairs=pairs)
    grp.submit([p[0].data_ptr() for p in parts], B)   # warm-up
    torch.cuda.synchronize()
    hs[0].shard_options(serial=True, profile=True, pairs=pairs)
    for s in range(1, args.steps + 1):
        grp.submit([p[s * B].data_ptr() for p in parts], B)
    torch.cuda.synchronize()
    per_rank = [h.shard_timing()[0] for h in hs]
    compute = [sum(v for k, v in t.items() if k not in EXCHANGE) for t in per_rank]
    # rank 0 alone on the GPU, pipelined (TSLAM_SHARD_SOLO | TSLAM_SHARD_PIPELINE): its front end
    # of batch s + 1 beside its back end of batch s on the driver's own streams, no exchange — the
    # per-GPU step of an N-GPU node whose exchange is hidden
    hs[0].shard_options(solo=True, pipeline=True, pairs=pairs)
    stream = torch.cuda.current_stream().cuda_stream
    grp.submit([p[0].data_ptr() for p in parts], B, [stream] * W)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(1, args.steps + 1):
        grp.submit([p[s * B].data_ptr() for p in parts], B, [stream] * W)
    torch.cuda.synchronize()
    solo_us = (time.perf_counter() - t0) / args.steps * 1e6
    sb, pr = hs[0].exchange_sizes()
    if pairs:   # rank 0: its camera of the partner's half + 1 frame; its pair's blocks of the other rig ranges of its half
        pb, hf = hs[0].pair_block_bytes(), B - B // 2 + 1
        sent = {"raw_images": hf * 640 * 400, "stream_blocks": hf * sb,
                "pair_blocks": (W // 2 - 1) * (B // W) * pb if len(rects) > 1 else 0, "pose_records": (B // W) * pr}
        largest = hf * (640 * 400 + sb)
    else:
        fr = B // W + 1   # frames a rank reads of each peer's cameras
        sent = {"raw_images": (W - 1) * fr * S * 640 * 400, "stream_blocks": (W - 1) * fr * S * sb,
                "pose_records": (B // W) * pr}
        largest = fr * S * (640 * 400 + sb)
    sent["total"] = sum(sent.values())
    sent["largest_to_one_peer"] = largest
    grp.close()
    for h in hs:
        h.close()
    out = {"world": W, "batch": B, "streams": C, "stereo_pairs": len(rects), "driver": "library (copy, serial)",
           "layout": "pair split (TSLAM_SHARD_PAIRS)" if pairs else "frame ranges",
           "us_per_step_per_rank": per_rank, "per_gpu_compute_us": max(compute),
           "per_gpu_compute_us_by_rank": compute, "bytes_sent_per_rank_per_step": sent,
           "rank0_pipelined_step_us": solo_us}
    if args.one_gpu:
        h = Handle(rects, cfg, max_batch=B)
        if len(rects) > 1:
            h.set_rig(E)
        fs, bs = torch.cuda.Stream(priority=-1), torch.cuda.Stream()

        def step(s):
            h.begin_batch(seq[s * B].data_ptr(), B)
            for st in ("rectify", "detect", "describe"):
                h.run_stage(st, fs.cuda_stream)
            for st in ("match", "pose"):
                h.run_stage(st, bs.cuda_stream)
            h.end_batch()

        step(0)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for s in range(1, args.steps + 1):
            step(s)
        torch.cuda.synchronize()
        out["one_gpu_step_us"] = (time.perf_counter() - t0) / args.steps * 1e6
        out["ratio_one_gpu_over_per_gpu"] = out["one_gpu_step_us"] / out["per_gpu_compute_us"]
        out["ratio_one_gpu_over_rank0_pipelined"] = out["one_gpu_step_us"] / solo_us
        h.close()
    line = json.dumps(out)
    print(line)
    if args.out:
        Path(args.out).write_text(line + "\n")


if __name__ == "__main__":
    main()
