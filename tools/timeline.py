"""Print a kernel timeline around one steady-state step from a rocprofv3 --kernel-trace CSV.

    python tools/timeline.py run_kernel_trace.csv [--anchor k_rectify_pyramid] [--nth 3]
"""
import argparse
import csv

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--anchor", default="k_rectify_pyramid")
ap.add_argument("--nth", type=int, default=3)
ap.add_argument("--span", type=int, default=2)
a = ap.parse_args()
rows = [r for r in csv.DictReader(open(a.trace)) if r["Kernel_Name"].startswith(("k_", "__amd"))]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
anc = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith(a.anchor + "(")]
i0, i1 = anc[a.nth], anc[min(a.nth + a.span, len(anc) - 1)]
t0 = int(rows[i0]["Start_Timestamp"])
for r in rows[i0:i1 + 1]:
    s = (int(r["Start_Timestamp"]) - t0) / 1000
    e = (int(r["End_Timestamp"]) - t0) / 1000
    print(f"{r['Kernel_Name'].split('(')[0][:26]:26s} q{r['Queue_Id']:>2} {s:9.1f} {e:9.1f} {e - s:8.1f}")
