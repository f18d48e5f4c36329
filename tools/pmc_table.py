"""Per-kernel table of rocprofv3 --pmc counters (averaged over dispatches), one or more run dirs.

usage: python tools/pmc_table.py DIR [DIR ...]
Derived columns: valu/wave, VALU busy % = SQ_INSTS_VALU * 2 cycles / (SIMDs * kernel cycles),
wait % = SQ_WAIT_ANY / SQ_WAVE_CYCLES (both quad-cycle counters).
"""
import collections
import csv
import sys

SIMDS = 1024
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for d in sys.argv[1:]:
    for r in csv.DictReader(open(d + "/run_counter_collection.csv")):
        k = r["Kernel_Name"].split("(")[0]
        if not k.startswith("k_"):
            continue
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[(d, k)].add(r["Dispatch_Id"])
for k, v in agg.items():
    n = max(len(disp[(d, k)]) for d in sys.argv[1:] if (d, k) in disp)
    m = {c: x / n for c, x in v.items()}
    waves = max(m.get("SQ_WAVES", 1), 1)
    cyc = m.get("GRBM_GUI_ACTIVE", 0) / 8
    busy = 100 * m.get("SQ_INSTS_VALU", 0) * 2 / SIMDS / cyc if cyc else 0
    wait = 100 * m.get("SQ_WAIT_ANY", 0) / max(m.get("SQ_WAVE_CYCLES", 1), 1)
    print(f"{k:18s} waves {waves:9.0f} valu/wave {m.get('SQ_INSTS_VALU', 0) / waves:7.0f} lds/wave {m.get('SQ_INSTS_LDS', 0) / waves:6.0f} "
          f"vmem/wave {m.get('SQ_INSTS_VMEM', 0) / waves:6.1f} VALU-busy {busy:5.1f}% wait {wait:5.1f}% "
          f"lds-conf {100 * m.get('SQ_LDS_BANK_CONFLICT', 0) / max(m.get('SQ_LDS_IDX_ACTIVE', 1), 1):5.1f}% kcyc {cyc / 1e3:7.0f}")
