"""Per-kernel SQ counter summary of a rocprofv3 --pmc run (SQ_WAVE_CYCLES/WAIT/ACTIVE are quad-cycles)."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1] + "/run_counter_collection.csv")))
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    k = r["Kernel_Name"].split("(")[0]
    if k.startswith("k_"):
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
cols = ["SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY"]
print(f"{'kernel':16s}" + "".join(f"{c[8:]:>14s}" for c in cols) + "  valu/wave  cyc/wave  wait%")
for k, d in agg.items():
    m = {c: sum(v) / len(v) for c, v in d.items()}
    w = max(m.get("SQ_WAVES", 1), 1)
    wc = m.get("SQ_WAVE_CYCLES", 0)
    print(f"{k:16s}" + "".join(f"{m.get(c, 0):14.4g}" for c in cols)
          + f"  {m.get('SQ_INSTS_VALU', 0) / w:9.0f} {4 * wc / w:9.0f} {100 * m.get('SQ_WAIT_ANY', 0) / max(wc, 1):6.1f}")
