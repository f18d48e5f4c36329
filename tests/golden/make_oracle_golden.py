"""Golden digests of the oracle's own outputs (first 3 frames of the seed-0 sequence).

The images are regenerated from the seed and not stored.  The fixture holds SHA-256 digests of:
- every integer stage: keypoints, descriptors and matches;
- every bit-exact floating stage: refined disparities and 3D correspondences.
It also holds the poses in full.  tests/test_golden_oracle.py recomputes these and compares, which
pins the specification against regressions.

    python tests/golden/make_oracle_golden.py
"""

from __future__ import annotations

import hashlib
import json
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "thor-slam_amd"), str(ROOT / "tests")]

N = 3


def digest(a) -> str:
    a = np.ascontiguousarray(a)
    return hashlib.sha256(a.tobytes() + str(a.dtype).encode() + str(a.shape).encode()).hexdigest()[:32]


def record(sc) -> dict:
    out = {"frames": digest(sc["frames"]), "per_frame": []}
    for i, r in enumerate(sc["oracle"]):
        cur = r["cur"]
        rec = {}
        for side in ("left", "right"):
            im = cur[side]
            v = im["valid"]
            rec[f"{side}_counts"] = list(map(int, im["counts"]))
            rec[f"{side}_kp"] = digest(np.stack([im["kp"][k][v] for k in ("x", "y", "level", "score", "angle")]))
            rec[f"{side}_desc"] = digest(im["desc"][v])
        rec["stereo"] = digest(cur["stereo"])
        rec["disp"] = digest(cur["disp"])
        rec["temporal"] = digest(cur["temporal"])
        rec["status"] = int(r["status"])
        rec["T"] = np.asarray(r["T"]).tolist()
        if i:
            c = r["corr"]
            rec["corr"] = digest(np.stack([c[k] for k in ("X", "Y", "Z", "du", "dv")]))
            rec["n_corr"] = int(c["X"].size)
            rec["best_hyp"] = int(r["best_hyp"])
            rec["n_inliers"] = int(r["n_inliers"])
        out["per_frame"].append(rec)
    return out


def main():
    from helpers import scenario

    data = {"seed0": record(scenario(seed=0, n=N)), "seed0_distorted": record(scenario(seed=0, n=2, distorted=True))}
    (HERE / "oracle_digest.json").write_text(json.dumps(data, indent=1))
    print("wrote", HERE / "oracle_digest.json")


if __name__ == "__main__":
    main()
