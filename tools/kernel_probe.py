"""Time single kernels back to back on resident data (profiling aid, not the bench).

    python tools/kernel_probe.py [--batch 256] [--kernels rectify_pyramid,detect,detect,detect]

Runs one full batch first (so every buffer holds real data), then launches the listed kernels in
order inside one batch and prints each launch's duration from HIP events on the launch stream.
Also times a device-to-device copy of the batch's pyramid slice as a bandwidth reference.
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
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--kernels", default="rectify_pyramid,detect,detect,detect,select,describe,describe")
    ap.add_argument("--width", type=int, default=640)
    ap.add_argument("--height", type=int, default=400)
    ap.add_argument("--features", type=int, default=2000)
    ap.add_argument("--ransac-counters", action="store_true",
                    help="print the per-block counters an instrumented k_ransac build leaves in qbest")
    ap.add_argument("--splits", type=int, default=0, help="RANSAC splits per frame (0: the library's choice)")
    args = ap.parse_args()
    import torch

    from bench import render_frames, triangle_indices
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
    if (args.width, args.height) == (640, 400):
        uniq = render_frames(0, 48, 8)
    else:
        uniq = src.render_stereo_sequence(16)
    frames = uniq[triangle_indices(2 * B, len(uniq))]
    dev = torch.from_numpy(frames).cuda()
    h = Handle([rect], HipSlamConfig(n_features=args.features), max_batch=B, ransac_splits=args.splits)
    stream = torch.cuda.current_stream()
    s = stream.cuda_stream
    h.submit(dev[:B].data_ptr(), B, s)
    h.submit(dev[B:].data_ptr(), B, s)
    torch.cuda.synchronize()
    import numpy as np

    print("te per camera x level:", h.frame_block("det_thr", 0, np.uint32).reshape(2, -1).tolist())
    h.begin_batch(dev[:B].data_ptr(), B)
    for name in args.kernels.split(","):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        h.run_kernel(name, s)
        e1.record(stream)
        torch.cuda.synchronize()
        print(f"{name:16s} {1000 * e0.elapsed_time(e1):9.1f} us")
    st = np.stack([h.frame_block("stats", i, np.int32)[:5] for i in range(0, B, max(1, B // 64))])
    ok = st[:, 0] == 0
    print("pose stats over %d sampled frames: tracked %d, correspondences n mean %.0f min %d max %d, "
          "RANSAC best count / n mean %.3f min %.3f, refined inliers / n mean %.3f" % (
              len(st), ok.sum(), st[:, 1].mean(), st[:, 1].min(), st[:, 1].max(),
              (st[:, 3] / np.maximum(st[:, 1], 1)).mean(), (st[:, 3] / np.maximum(st[:, 1], 1)).min(),
              (st[:, 2] / np.maximum(st[:, 1], 1)).mean()))
    if args.ransac_counters:
        names = ["break", "visited", "nan", "pre_drop", "superchunks", "scan_drop", "complete", "n"]
        cnt = np.stack([h.frame_block("qbest", i, np.uint32)[:8] for i in range(B)]).astype(np.int64)
        print("k_ransac counters per block: mean " + " ".join("%s %.1f" % (k, v) for k, v in zip(names, cnt.mean(0))))
        print("  max " + " ".join("%s %d" % (k, v) for k, v in zip(names, cnt.max(0))))
        top = np.argsort(-cnt[:, 4])[:5]
        print("  slowest blocks (superchunks):", [(int(i), cnt[i].tolist()) for i in top])
    h.end_batch()
    # bandwidth reference: copy the pyramid slice of B frames (read + write)
    import ctypes

    ptr, total, per = h.buffer_info("pyramid") if hasattr(h, "buffer_info") else (None, None, None)
    if ptr is not None:
        nbytes = per * B
        a = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
        b = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            b.copy_(a)
            e1.record(stream)
            torch.cuda.synchronize()
            us = 1000 * e0.elapsed_time(e1)
            print(f"copy {nbytes / 1e6:.0f} MB  {us:9.1f} us  {2 * nbytes / us / 1e3:.0f} GB/s")
    h.close()


if __name__ == "__main__":
    main()
