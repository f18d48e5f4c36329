"""LDS bank-conflict degree of the rotated-BRIEF reads in k_describe for candidate tile pitches.

A wave reads one byte per lane at (py + 18) * pitch + px + 18 for 64 consecutive pattern pairs;
the LDS serves one dword per bank per cycle, so a wave's read takes as many cycles as the most
distinct dwords that share a bank.  Prints the average over the 30 bins x 4 lane groups x the 4
byte alignments of the keypoint, for the first and the second point of each pair.
"""

from __future__ import annotations

import re
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]


def table() -> np.ndarray:
    src = (ROOT / "thor-slam_amd" / "csrc" / "tslam_tables.h").read_text()
    m = re.search(r"TSLAM_BRIEF_TABLE\[[^\]]*\]\s*=\s*\{([^}]*)\}", src, re.S)
    return np.array([int(x, 0) for x in re.findall(r"0x[0-9a-fA-F]+|\d+", m.group(1))], dtype=np.int64).reshape(30, 256)


def degree(pitch: int, x: np.ndarray, y: np.ndarray) -> float:
    tot = []
    for b in range(30):
        for j in range(4):
            for shift in range(4):
                dw = ((y[b, 64 * j:64 * j + 64] + 18) * pitch + x[b, 64 * j:64 * j + 64] + 18 + shift) // 4
                banks = np.bincount(np.unique(dw) % 64, minlength=64)
                tot.append(banks.max())
    return float(np.mean(tot))


def main() -> None:
    t = table()
    s8 = lambda v: ((v & 0xFF) ^ 0x80) - 0x80   # noqa: E731
    px, py, qx, qy = s8(t), s8(t >> 8), s8(t >> 16), s8(t >> 24)
    for pitch in [int(a) for a in sys.argv[1:]] or [192, 196, 200, 208, 224, 240, 256]:
        print(f"pitch {pitch}: first point {degree(pitch, px, py):.2f}, second point {degree(pitch, qx, qy):.2f}")


if __name__ == "__main__":
    main()
