"""How well two kernel groups share the GPU (profiling aid, not the bench).

    python tools/overlap_probe.py

Two handles hold the same resident C2 batch; for each pair (X, Y) it times X alone, Y alone and
X on one stream beside Y on another (both released by one event), HIP events throughout.  A
concurrent time well under alone(X) + alone(Y) means the pipelined step gains by overlapping
those groups.
"""

from __future__ import annotations

import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for p in (ROOT, ROOT / "thor-slam_amd"):
    sys.path.insert(0, str(p))


def main() -> None:
    import torch

    from bench import render_frames, triangle_indices
    from thor_slam_amd._lib import Handle
    from thor_slam_amd.calib import extract_cameras, stereo_pairs, stereo_rectify
    from thor_slam_amd.camera.rig import CameraRig
    from thor_slam_amd.params import HipSlamConfig
    from thor_slam_amd.synthetic import SyntheticStereoSource

    src = SyntheticStereoSource(seed=0)
    cams = extract_cameras(CameraRig([src]).calibration, 2)
    (li, ri), = stereo_pairs(cams)
    rect = stereo_rectify(cams[li], cams[ri])
    import os

    B = int(os.environ.get("PROBE_BATCH", "1024"))
    frames = render_frames(0, 48, 8)[triangle_indices(2 * B, 48)]
    dev = torch.from_numpy(frames).cuda()
    hs = [Handle([rect], HipSlamConfig(), max_batch=B) for _ in range(2)]
    s0 = torch.cuda.current_stream()
    for h in hs:
        h.submit(dev[:B].data_ptr(), B, s0.cuda_stream)
        h.submit(dev[B:].data_ptr(), B, s0.cuda_stream)
    torch.cuda.synchronize()
    sa, sb = torch.cuda.Stream(priority=-1), torch.cuda.Stream()   # sa: the high-priority front stream of the bench

    def run(h, group, st):
        h.begin_batch(dev[:B].data_ptr(), B)
        for k in group:
            h.run_kernel(k, st.cuda_stream)
        h.end_batch()

    def timed(parts):
        go = torch.cuda.Event()
        go.record(s0)
        ends = []
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record(s0)
        for h, group, st in parts:
            st.wait_event(go)
            run(h, group, st)
            e = torch.cuda.Event(enable_timing=True)
            e.record(st)
            ends.append(e)
        for e in ends:
            s0.wait_event(e)
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record(s0)
        torch.cuda.synchronize()
        return 1000 * e0.elapsed_time(e1)

    pairs = [(["detect"], ["match", "match_refine", "pose", "chain"]),
             (["select", "describe"], []),
             (["detect"], ["match", "match_refine"]),
             (["select", "describe"], ["pose", "chain"]),
             (["describe"], ["pose", "chain"]),
             (["detect", "select"], ["match", "match_refine"]),
             (["describe"], ["match", "match_refine", "pose", "chain"])]
    for X, Y in pairs:
        res = []
        for _ in range(3):
            a = timed([(hs[0], X, sa)])
            b = timed([(hs[1], Y, sb)]) if Y else 0.0
            c = timed([(hs[0], X, sa), (hs[1], Y, sb)]) if Y else a
            res.append((a, b, c))
        a, b, c = (min(r[i] for r in res) for i in range(3))
        print(f"{'+'.join(X):16s} {a:7.1f} | {'+'.join(Y):34s} {b:7.1f} | together {c:7.1f} "
              f"(sum {a + b:7.1f}, saves {100 * (1 - c / (a + b)):4.1f} %)")
    for h in hs:
        h.close()


if __name__ == "__main__":
    main()
