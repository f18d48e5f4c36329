"""The default drop-in path (bench.py default_config_bench) on the C2 lap with the loop trace on:
frames/s, loops, and on a failing loop job the failing span solve's inputs saved to
gpurun_out/loop_probe_fail.npz.   python tools/loop_probe.py [--frames 512] [--kind c2]"""

from __future__ import annotations

import argparse
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
for p in (ROOT, ROOT / "thor-slam_amd"):
    sys.path.insert(0, str(p))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=512)
    ap.add_argument("--kind", default="c2")
    ap.add_argument("--profile", action="store_true", help="cProfile the timed loop (top entries by own time)")
    ap.add_argument("--trace", type=int, default=1, help="record the loop trace (0: as deployed)")
    ap.add_argument("--sort", default="tottime", help="cProfile sort key (tottime, cumulative)")
    ap.add_argument("--callees", default="", help="also print the callees of functions matching this name")
    args = ap.parse_args()
    import bench
    from thor_slam_amd.camera import CameraRig, Extrinsics
    from thor_slam_amd.camera.types import IMUExtrinsics
    from thor_slam_amd.slam.hip_engine import HipSlamEngine
    from thor_slam_amd.synthetic import DRB_TO_RDF
    import json

    names = bench.C3_NAMES if args.kind == "c3" else bench.C3_NAMES[:1]
    items = [(q, i, c) for q in range(len(names)) for i in range(bench.LAP) for c in (0, 1)]
    w = bench.usable_cpus()
    chunks = [items[k::w] for k in range(w) if items[k::w]]
    frames = {nm: np.empty((bench.LAP, 2, 400, 640), np.uint8) for nm in names}
    from concurrent.futures import ProcessPoolExecutor

    with ProcessPoolExecutor(max_workers=len(chunks)) as ex:
        for ch, imgs in zip(chunks, ex.map(bench._render_lap_chunk, [(names, ch) for ch in chunks])):
            for (q, i, c), img in zip(ch, imgs):
                frames[names[q]][i, c] = img
    joints = json.loads(bench.JOINTS.read_text())
    srcs = bench._lap_sources(names, frames)
    base_T_imu = np.array(joints[names[0]]) @ DRB_TO_RDF
    rig = CameraRig(srcs, rig_extrinsics={nm: Extrinsics.from_4x4_matrix(np.array(joints[nm])) for nm in names},
                    imu_source=names[0], imu_extrinsics=IMUExtrinsics(names[0], Extrinsics.from_4x4_matrix(base_T_imu)))
    rig.start()
    sets = [rig.get_synchronized_frames() for _ in range(args.frames)]
    eng = HipSlamEngine(num_cameras=2 * len(names))
    eng.initialize(rig.calibration)
    if args.trace:
        eng._loop.trace = {}
    for fs in sets[:64]:   # warm-up (kernels, loop jobs, scratch)
        eng.process_frames(fs)
    eng.settle()
    eng.reset()
    prof = None
    if args.profile:
        import cProfile

        prof = cProfile.Profile()
        prof.enable()
    t0 = time.perf_counter()
    try:
        for i, fs in enumerate(sets):
            eng.process_frames(fs)
        eng.flush()
    except RuntimeError as exc:
        lp = eng._loop
        print(f"failed at frame {i}: {exc}")
        for f in lp.failures:
            T, e, m, inf = f["args"]
            Path("gpurun_out").mkdir(exist_ok=True)
            np.savez(f"gpurun_out/loop_probe_fail_{args.kind}.npz", T=T, edges=e, meas=m, info=inf, ver_T=f["ver"]["T"],
                     ver_stats=f["ver"]["stats"], qcpc=np.array([f["q"], f["c"], f["pc"], f["idx"], f["g"]]))
            print("failure", {k: f[k] for k in ("idx", "g", "q", "c", "pc", "error")}, "finite:", np.isfinite(T).all(),
                  np.isfinite(m).all(), "span", len(T), "edges", len(e))
            # the same inputs again on the device, twice (deterministic?) and against the oracle
            from oracle import numpy_loop as L

            for _ in range(2):
                try:
                    r = eng.handle.pose_graph(T, e, m, inf, eng._config.pg_iters)
                    print("device re-solve finite", np.isfinite(r["T"]).all(), "cost", r["cost"])
                except RuntimeError as e2:
                    print("device re-solve:", e2)
            o = L.optimize(T, e, m, inf, eng._config.pg_iters)
            print("oracle solve finite", np.isfinite(o["T"]).all(), "cost", o["cost"], "steps", o["steps"])
        raise
    dt = time.perf_counter() - t0
    if prof is not None:
        import pstats

        prof.disable()
        st = pstats.Stats(prof).sort_stats(args.sort)
        st.print_stats(30)
        if args.callees:
            st.print_callees(args.callees)
    lp = eng._loop
    print(f"{args.kind}: {args.frames / dt:.0f} frames/s, {len(lp.frames)} keyframes, {len(lp.loops)} loops, "
          f"state {eng.get_tracking_state().name}, async {eng._async}, imu {eng._imu is not None}")
    eng.shutdown()


if __name__ == "__main__":
    main()
