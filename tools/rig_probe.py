"""Back-end kernels of one rank's frame range, timed alone (profiling aid, not the bench).

    [TSLAM_LIBRARY=exp/libtslam_rigstamps.so] python tools/rig_probe.py [--batch 32] [--names 4]

The C3 bracket rig (4 stereo sources) on one handle with max_batch = --batch (32 = the frame range
one of 8 ranks solves of a 256-frame batch): two full batches, then match, match_refine, pose, rig
and chain launched alone inside a third batch, each timed with HIP events (3 repetitions).  With an
experiment build compiled with -DTS_RIG_STAMPS, k_rig_pose prints its phase durations.
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
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--names", type=int, default=4)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    import torch

    from bench import RIG_SOURCES, render_rig_frames, rig_setup, triangle_indices
    from thor_slam_amd._lib import Handle
    from thor_slam_amd.params import HipSlamConfig

    names = RIG_SOURCES[:args.names]
    _, cams, pairs, rects, E = rig_setup(names)
    C, B = 2 * len(rects), args.batch
    uniq = render_rig_frames(names, 24, 0, C, 8)
    seq = torch.from_numpy(uniq[triangle_indices(3 * B, 24)]).cuda()
    h = Handle(rects, HipSlamConfig(), max_batch=B)
    h.set_rig(E)
    st = torch.cuda.current_stream()
    for s in range(2):
        h.submit(seq[s * B].data_ptr(), B, st.cuda_stream)
    torch.cuda.synchronize()
    kern = ["match", "match_refine", "pose", "rig", "chain"]
    us = {k: 0.0 for k in kern}
    for r in range(args.reps):
        h.begin_batch(seq[2 * B].data_ptr(), B)
        for k in ("rectify_pyramid", "detect", "select", "describe"):
            h.run_kernel(k, st.cuda_stream)
        evs = []
        for k in kern:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            if k == "rig":
                h.run_rig(st.cuda_stream)
            else:
                h.run_kernel(k, st.cuda_stream)
            e1.record(st)
            evs.append((k, e0, e1))
        h.end_batch()
        torch.cuda.synchronize()
        for k, e0, e1 in evs:
            us[k] += e0.elapsed_time(e1) * 1e3 / args.reps
    h.close()
    line = json.dumps({"batch": B, "pairs": len(rects), "us_alone": us})
    print(line, flush=True)
    if args.out:
        Path(args.out).write_text(line + "\n")


if __name__ == "__main__":
    main()
