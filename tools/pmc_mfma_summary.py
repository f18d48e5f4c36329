"""Per-kernel FP64 MFMA summary of a rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU SQ_WAVES
pass (tools/prof_c4.sh): counters averaged per launch; MOPS are in units of 512 FP64 flops, so
mfma_f64_flops_per_launch = 512 * SQ_INSTS_VALU_MFMA_MOPS_F64.

usage: python tools/pmc_mfma_summary.py PMC_DIR OUT_JSON [NOTE]
"""

import collections
import csv
import json
import sys
from pathlib import Path


def main() -> None:
    d, out = Path(sys.argv[1]), Path(sys.argv[2])
    note = sys.argv[3] if len(sys.argv) > 3 else ""
    rows = [r for fp in sorted(d.rglob("*counter_collection.csv")) for r in csv.DictReader(open(fp))]
    per = collections.defaultdict(lambda: collections.defaultdict(float))   # kernel -> dispatch -> counter sums
    for r in rows:
        k = r["Kernel_Name"].split("(")[0]
        if k.startswith("k_"):
            per[(k, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for (k, _), cs in per.items():
        for c, v in cs.items():
            agg[k][c].append(v)
    res = {}
    for k, cs in agg.items():
        e = {c: sum(v) / len(v) for c, v in cs.items()}
        e["launches"] = max(len(v) for v in cs.values())
        e["mfma_f64_flops_per_launch"] = 512.0 * e.get("SQ_INSTS_VALU_MFMA_MOPS_F64", 0.0)
        res[k] = e
    out.write_text(json.dumps({"note": note, "kernels": res}, indent=1))
    for k in ("k_ba_schur", "k_pg_syrk"):
        if k in res:
            print(k, {c: round(v, 1) for c, v in res[k].items()})


if __name__ == "__main__":
    main()
