"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into per-kernel HBM bytes per launch.

Correction (MI355X_MICROARCH.md §HBM, cdna_hip_programming.md §7): counters are in KiB;
FETCH_SIZE reports half the bytes of a wide coalesced read on gfx950.  The doubling holds only for
16-byte-per-lane streaming reads, so it is applied per kernel: to the kernels whose reads are
such streams (WIDE_READS: rectify's 16-B row loads, detect's and describe's LDS-DMA tiles,
the exchange gathers) traffic = (2 * FETCH_SIZE + WRITE_SIZE) * 1024; every other kernel
(gathers, scalar loads, byte reads) is reported uncorrected, (FETCH_SIZE + WRITE_SIZE) * 1024.
Each kernel's entry names the correction it got.

An optional third pass (``--sq DIR``: SQ_INSTS_VALU, SQ_WAVES) adds the VALU wave-instructions
per launch, the numerator of the VALU-issue roofline in bench.py (peak: 256 CUs x 4 SIMD-32 x
2.4 GHz / 2 cycles per wave64 instruction = 1.2288e12 wave-instructions/s, MI355X_MICROARCH.md
"Execution model").

usage: python tools/pmc_summary.py FETCH_DIR WRITE_DIR OUT_JSON [--batch B] [--sq SQ_DIR]
"""

import collections
import csv
import json
import sys
from pathlib import Path


def load(d, counter=None):
    files = sorted(Path(d).rglob("*counter_collection.csv"))
    if not files:
        raise SystemExit(f"no *counter_collection.csv under {d}")
    rows = [r for fp in files for r in csv.DictReader(open(fp))]
    agg = collections.defaultdict(list)
    for r in rows:
        if counter is None or r["Counter_Name"] == counter:
            agg[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


# kernels whose HBM reads are 16-byte-per-lane coalesced streams (the FETCH_SIZE halving applies)
WIDE_READS = {"k_rectify_pyramid", "k_detect", "k_detect_fallback", "k_describe", "k_stream_blocks", "k_tsdf_integrate"}


def main():
    fetch, write, out = sys.argv[1], sys.argv[2], sys.argv[3]
    batch = int(sys.argv[sys.argv.index("--batch") + 1]) if "--batch" in sys.argv else None
    sq = sys.argv[sys.argv.index("--sq") + 1] if "--sq" in sys.argv else None
    f, w = load(fetch), load(write)
    valu = load(sq, "SQ_INSTS_VALU") if sq else {}
    waves = load(sq, "SQ_WAVES") if sq else {}
    res = {}
    for k in sorted(set(f) | set(w)):
        if not k.startswith("k_"):
            continue
        fk, wk = f.get(k, 0.0), w.get(k, 0.0)
        wide = k.split("<")[0] in WIDE_READS
        res[k] = {"FETCH_SIZE_KiB": fk, "WRITE_SIZE_KiB": wk,
                  "hbm_bytes_per_launch": ((2 if wide else 1) * fk + wk) * 1024.0,
                  "hbm_bytes_per_launch_uncorrected": (fk + wk) * 1024.0,
                  "traffic_note": ("(2 FETCH_SIZE + WRITE_SIZE) KiB: 16-B/lane streaming reads, gfx950 FETCH_SIZE halving"
                                   if wide else "(FETCH_SIZE + WRITE_SIZE) KiB, uncorrected: gathers / narrow reads")}
        if k in valu:
            res[k]["valu_insts_per_launch"] = valu[k]
            res[k]["waves_per_launch"] = waves.get(k)
    Path(out).write_text(json.dumps({"batch_frames": batch, "kernels": res}, indent=1))
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
