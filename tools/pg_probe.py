"""Time the device pose-graph solve (tslam_pose_graph) on random keyframe graphs (profiling aid).

    python tools/pg_probe.py [--nodes 64,256,1024] [--iters 8] [--reps 3]

Each graph is a chain of N keyframes plus loop edges, either SLAM-like (the newest keyframes
closing on old ones: a thin matrix profile) or N/20 random long-range edges (a wide one); prints the wall time of one solve and
the algorithmic FP64 flops of its Cholesky factorisations (np^3/3 per iteration, np = 6(N-1)
padded to 32), whose trailing updates run on the FP64 matrix cores (k_pg_syrk).
"""

from __future__ import annotations

import argparse
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
for p in (ROOT, ROOT / "thor-slam_amd"):
    sys.path.insert(0, str(p))


def graph(rng, N, slam_like=False):
    from oracle import numpy_loop as L

    gt = [np.eye(4)]
    for _ in range(1, N):
        gt.append(gt[-1] @ L.se3_exp(np.r_[rng.normal(0, 0.1, 3), rng.normal(0, 0.05, 3)]))
    if slam_like:   # loop edges from the newest keyframes back to old ones (a revisit)
        loops = [(int(a), N - 1 - i) for i, a in enumerate(rng.integers(0, N // 4, max(1, N // 100)))]
    else:           # worst case for the profile: random long-range edges
        loops = [(int(a), int(b)) for a, b in zip(rng.integers(0, N // 2, N // 20), rng.integers(N // 2, N, N // 20))]
    edges = [(i, i + 1) for i in range(N - 1)] + loops
    Z = np.array([L.inv_se3(gt[i]) @ gt[j] @ L.se3_exp(rng.normal(0, 0.002, 6)) for i, j in edges])
    T0 = [np.eye(4)]
    for k in range(N - 1):
        T0.append(T0[-1] @ Z[k])
    info = np.array([L.loop_information(0.01, 0.005)] * len(edges))
    return np.array(T0), np.array(edges), Z, info


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", default="64,256,1024")
    ap.add_argument("--iters", type=int, default=8)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import torch  # noqa: F401  (HIP runtime first, see _lib.load_library)

    from thor_slam_amd._lib import Handle
    from thor_slam_amd.calib import extract_cameras, stereo_pairs, stereo_rectify
    from thor_slam_amd.camera.rig import CameraRig
    from thor_slam_amd.params import HipSlamConfig
    from thor_slam_amd.synthetic import SyntheticStereoSource

    src = SyntheticStereoSource(seed=0)
    cams = extract_cameras(CameraRig([src]).calibration, 2)
    (li, ri), = stereo_pairs(cams)
    h = Handle([stereo_rectify(cams[li], cams[ri])], HipSlamConfig(), max_batch=1)
    rng = np.random.default_rng(0)
    for N, kind in [(int(x), k) for x in args.nodes.split(",") for k in ("slam-like", "random-loops")]:
        T0, edges, Z, info = graph(rng, N, kind == "slam-like")
        h.pose_graph(T0, edges, Z, info, args.iters)   # warm-up (allocations)
        ts = []
        for _ in range(args.reps):
            t = time.perf_counter()
            res = h.pose_graph(T0, edges, Z, info, args.iters)
            ts.append(time.perf_counter() - t)
        n = 6 * (N - 1)
        npad = (n + 31) // 32 * 32
        flops = args.iters * npad ** 3 / 3.0
        best = min(ts)
        print(f"{kind:12s} nodes {N:5d} edges {len(edges):5d} unknowns {n:5d}: {best * 1e3:8.2f} ms per solve "
              f"({args.iters} iterations), Cholesky {flops / best / 1e12:.3f} TFLOP/s, cost {res['cost']:.4g}", flush=True)
    h.close()


if __name__ == "__main__":
    main()
