"""Profile the host boundary at B = 1 (HipSlamEngine.process_frames over CameraRig frame sets from
host memory, as bench.py's boundary leg): frames/s, then a cProfile of the same loop (top entries by
own time).   python tools/boundary_probe.py [--frames 600] [--batch 1]"""

from __future__ import annotations

import argparse
import cProfile
import pstats
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for p in (ROOT, ROOT / "thor-slam_amd"):
    sys.path.insert(0, str(p))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=600)
    ap.add_argument("--batch", type=int, default=1)
    args = ap.parse_args()
    import bench
    from thor_slam_amd.camera.rig import CameraRig
    from thor_slam_amd.params import HipSlamConfig
    from thor_slam_amd.slam.hip_engine import HipSlamEngine
    from thor_slam_amd.synthetic import SyntheticStereoSource

    src = SyntheticStereoSource(seed=0, n_frames=48)
    uniq = src.render_stereo_sequence(24)
    rep = bench._ReplaySource(src.name, uniq, src.get_intrinsics(), src.get_extrinsics())
    rig = CameraRig([rep])
    rig.start()
    sets = [rig.get_synchronized_frames() for _ in range(args.frames)]
    eng = HipSlamEngine(num_cameras=2, config=HipSlamConfig(batch_size=args.batch, enable_loop_closure=False))
    eng.initialize(rig.calibration)
    for s in sets[:20]:
        eng.process_frames(s)
    eng.flush()
    t0 = time.perf_counter()
    for s in sets:
        eng.process_frames(s)
    eng.flush()
    dt = time.perf_counter() - t0
    print(f"B={args.batch}: {args.frames / dt:.0f} frames/s ({dt / args.frames * 1e6:.0f} us per frame)")
    prof = cProfile.Profile()
    prof.enable()
    for s in sets:
        eng.process_frames(s)
    eng.flush()
    prof.disable()
    pstats.Stats(prof).sort_stats("tottime").print_stats(25)
    eng.shutdown()


if __name__ == "__main__":
    main()
