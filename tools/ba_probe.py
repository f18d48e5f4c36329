"""Time the A8 local BA stage at config C4 (profiling aid, not the bench).

    python tools/ba_probe.py [--batch 50] [--width 1280 --height 800 --features 4000 --window 10]

Submits --warm batches to fill the keyframe window, then runs --reps batches stage by stage and
prints the front end's and the BA stage's durations (HIP events on the launch stream), the host
time the BA stage call takes per keyframe, and the last solve's observation / landmark counts.
"""

from __future__ import annotations

import argparse
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for p in (ROOT, ROOT / "thor-slam_amd"):
    sys.path.insert(0, str(p))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=50)
    ap.add_argument("--width", type=int, default=1280)
    ap.add_argument("--height", type=int, default=800)
    ap.add_argument("--features", type=int, default=4000)
    ap.add_argument("--window", type=int, default=10)
    ap.add_argument("--interval", type=int, default=5)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--unique", type=int, default=24)
    ap.add_argument("--graph", type=int, default=1, help="tslam_ba_graph: 1 graph replays, 0 direct launches")
    ap.add_argument("--warm", type=int, default=4, help="batches submitted before the measured ones")
    ap.add_argument("--reps", type=int, default=4, help="measured batches (stage by stage, HIP events)")
    args = ap.parse_args()
    import numpy as np
    import torch

    from bench import triangle_indices
    from thor_slam_amd._lib import Handle
    from thor_slam_amd.calib import extract_cameras, stereo_pairs, stereo_rectify
    from thor_slam_amd.camera.rig import CameraRig
    from thor_slam_amd.params import HipSlamConfig
    from thor_slam_amd.synthetic import SyntheticStereoSource

    src = SyntheticStereoSource(seed=0, width=args.width, height=args.height)
    cams = extract_cameras(CameraRig([src]).calibration, 2)
    (li, ri), = stereo_pairs(cams)
    rect = stereo_rectify(cams[li], cams[ri])
    B = args.batch
    uniq = src.render_stereo_sequence(args.unique)
    n_b = args.warm + args.reps
    frames = np.ascontiguousarray(uniq[triangle_indices(n_b * B, len(uniq))])
    dev = torch.from_numpy(frames).cuda()
    cfg = HipSlamConfig(n_features=args.features, ba_window=args.window, ba_kf_interval=args.interval,
                        ba_iters=args.iters)
    h = Handle([rect], cfg, max_batch=B)
    h.ba_graph(bool(args.graph))
    stream = torch.cuda.current_stream()
    s = stream.cuda_stream
    for b in range(args.warm):   # fills the window (and, with graphs, captures the chain shapes)
        h.submit(dev[b * B:].data_ptr(), B, s)
    torch.cuda.synchronize()
    import time

    fe_ms, ba_ms, host_ms, n_kf = [], [], [], 0
    for b in range(args.warm, n_b):
        h.begin_batch(dev[b * B:].data_ptr(), B)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        ev[0].record(stream)
        for st in ("rectify", "detect", "describe", "match", "pose"):
            h.run_stage(st, s)
        ev[1].record(stream)
        t0 = time.perf_counter()
        h.run_stage("ba", s)
        host_ms.append(1e3 * (time.perf_counter() - t0))
        ev[2].record(stream)
        h.end_batch()
        torch.cuda.synchronize()
        fe_ms.append(ev[0].elapsed_time(ev[1]))
        ba_ms.append(ev[1].elapsed_time(ev[2]))
        n_kf += len([g for g in range(b * B, (b + 1) * B) if g % args.interval == 0])
    fe, ba, host = np.mean(fe_ms), np.sum(ba_ms), np.sum(host_ms)
    win = h.ba_read(0)
    print(f"front end   {fe:8.3f} ms  ({B} frames, {1000 * fe / B:.1f} us/frame)")
    print(f"local BA    {ba / args.reps:8.3f} ms per batch ({n_kf} keyframes over {args.reps} batches, "
          f"{ba / max(n_kf, 1):.4f} ms/keyframe); host issue {host / max(n_kf, 1) * 1e3:.1f} us/keyframe "
          f"(graph={args.graph})")
    print(f"last solve  n_obs={win['n_obs']} n_lm={win['n_lm']} ok={win['ok']} window={sorted(win['frames'].tolist())}")
    h.close()


if __name__ == "__main__":
    main()
