"""The sharded rig's phases in the one-process rehearsal (profiling aid, not the bench).

    python tools/shard_probe.py [--world 8] [--batch 256] [--names 4]

All ranks of a LocalShardedRig on this GPU, one stream: every phase of every rank timed with HIP
events (kernels by name, raw staging, stream-block packing, the device copies standing in for the
RCCL all-to-all and all-gather, the imports that rectify the remote raw images).  Prints per-step
microseconds summed over the ranks and per rank, the bytes one rank sends per step, and the
per-GPU compute of an N-GPU run (the sum of one rank's phases without the copies), which bounds
the N-GPU step from below when the exchange is hidden.
"""

from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for p in (ROOT, ROOT / "thor-slam_amd"):
    sys.path.insert(0, str(p))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--names", type=int, default=4, help="stereo sources of the bracket rig (2 streams each)")
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    import torch

    from bench import RIG_SOURCES, render_rig_frames, rig_setup, triangle_indices
    from thor_slam_amd.params import HipSlamConfig
    from thor_slam_amd.shard import LocalShardedRig, StageTimer

    names = RIG_SOURCES[:args.names]
    _, cams, pairs, rects, E = rig_setup(names)
    C, B = 2 * len(rects), args.batch
    uniq = render_rig_frames(names, 24, 0, C, 8)
    seq = torch.from_numpy(uniq[triangle_indices((args.steps + 1) * B, 24)]).cuda()
    rig = LocalShardedRig(rects, HipSlamConfig(), world=args.world, batch=B, base_T_rect=E if len(rects) > 1 else None)
    st = torch.cuda.current_stream()
    rig.step(seq[:B], st)   # warm-up
    timer = StageTimer()
    timer.stream = st
    for s in range(1, args.steps + 1):
        rig.step(seq[s * B:(s + 1) * B], st, timer)
    torch.cuda.synchronize()
    tot = {k: sum(a.elapsed_time(b) for a, b in v) * 1e3 / args.steps for k, v in timer.spans.items()}
    W = args.world
    per_rank = {k: v / W for k, v in tot.items()}
    rk = rig.ranks[0]
    S, fr = rig.plan.streams_per_rank, rig.plan.recv_frames
    sent = {"raw_images": (W - 1) * fr * S * rk.img_bytes, "stream_blocks": (W - 1) * fr * S * rk.block,
            "pose_records": rig.plan.frames_per_rank * rk.record}
    compute = sum(v for k, v in per_rank.items() if k not in ("exchange", "pose_gather"))
    out = {"world": W, "batch": B, "streams": C, "stereo_pairs": len(rects), "us_per_step_all_ranks": tot,
           "us_per_step_per_rank": per_rank, "per_gpu_compute_us": compute,
           "bytes_sent_per_rank_per_step": sent, "bytes_sent_total": sum(sent.values())}
    line = json.dumps(out)
    print(line)
    if args.out:
        Path(args.out).write_text(line + "\n")


if __name__ == "__main__":
    main()
