"""GPU busy / overlap over steady-state steps of a rocprofv3 --kernel-trace CSV of bench.py:
the span of `steps` consecutive steps (anchored on k_rectify_pyramid launches), the time any kernel
runs, the time two or more run together, and the idle gaps by the kernel that follows them.

    python tools/timeline_busy.py run_kernel_trace.csv [--first 4] [--steps 4]
"""
import argparse
import collections
import csv

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--first", type=int, default=4)
ap.add_argument("--steps", type=int, default=4)
a = ap.parse_args()
rows = [r for r in csv.DictReader(open(a.trace))]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rect = [int(r["Start_Timestamp"]) for r in rows if r["Kernel_Name"].startswith("k_rectify_pyramid")]
t0, t1 = rect[a.first], rect[a.first + a.steps]
iv = [(max(int(r["Start_Timestamp"]), t0), min(int(r["End_Timestamp"]), t1), r["Kernel_Name"].split("(")[0])
      for r in rows if int(r["End_Timestamp"]) > t0 and int(r["Start_Timestamp"]) < t1]
ev = []
for s, e, n in iv:
    ev += [(s, 1, n), (e, -1, n)]
ev.sort(key=lambda x: (x[0], x[1]))
c, last, busy, two = 0, t0, 0, 0
gaps = collections.Counter()
for t, d, n in ev:
    if c >= 1:
        busy += t - last
    if c >= 2:
        two += t - last
    if c == 0 and d == 1 and t > last:
        gaps[n] += t - last
    c += d
    last = t
span = t1 - t0
print(f"{a.steps} steps: span {span / 1e3:.0f} us ({span / 1e3 / a.steps:.0f} per step), any kernel "
      f"{100 * busy / span:.1f} %, >= 2 kernels {100 * two / span:.1f} %, idle {100 * (1 - busy / span):.1f} %")
for n, g in gaps.most_common(8):
    print(f"  idle before {n:24s} {g / 1e3 / a.steps:8.1f} us per step")
