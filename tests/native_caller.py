"""The gcc-built native caller of the C-ABI (tests/c/rig_from_calib.c) and its file formats."""

from __future__ import annotations

import subprocess
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
SRC = ROOT / "tests" / "c" / "rig_from_calib.c"
LIB_DIR = ROOT / "thor-slam_amd" / "thor_slam_amd"
EXE = ROOT / "tests" / "c" / "build" / "rig_from_calib"


def build() -> Path:
    """Compile the caller with gcc against include/tslam.h and the in-tree libtslam_hip.so."""
    deps = (SRC, ROOT / "include" / "tslam.h")   # the caller bakes in the header's struct layouts
    if not EXE.exists() or EXE.stat().st_mtime < max(d.stat().st_mtime for d in deps):
        EXE.parent.mkdir(parents=True, exist_ok=True)
        subprocess.run(["gcc", "-O2", "-Wall", "-Werror", "-std=c11", f"-I{ROOT / 'include'}", str(SRC), "-o", str(EXE),
                        f"-L{LIB_DIR}", "-ltslam_hip", f"-Wl,-rpath,{LIB_DIR}"], check=True)
    return EXE


def write_calib(cams: list, path: Path) -> None:
    """calib.txt: one CameraConfig per line (17 significant digits: doubles read back exactly)."""
    lines = []
    for c in cams:
        intr = c.intrinsics
        d = np.zeros(14)
        co = np.asarray(intr.coeffs, dtype=np.float64).flatten()[:14]
        d[:len(co)] = co
        vals = list(np.asarray(intr.matrix, dtype=np.float64).reshape(9)) + list(d) + \
            list(c.extrinsics.to_4x4_matrix().reshape(16))
        lines.append(f"{c.source_name} {int(c.cam_idx)} {int(intr.width)} {int(intr.height)} {len(co)} " +
                     " ".join(f"{float(v):.17g}" for v in vals))
    Path(path).write_text("\n".join(lines) + "\n")


def read_maps(path: Path, pairs: int, width: int, height: int) -> list[dict]:
    """Output of ``rig_from_calib maps``."""
    raw = Path(path).read_bytes()
    cells = width * height * 2
    out, o = [], 0
    for _ in range(pairs):
        lr = np.frombuffer(raw, np.int32, 2, o); o += 8
        sc = np.frombuffer(raw, np.float64, 5, o); o += 40
        base = np.frombuffer(raw, np.float64, 16, o).reshape(4, 4); o += 128
        ml = np.frombuffer(raw, np.int32, cells, o).reshape(height, width, 2); o += 4 * cells
        mr = np.frombuffer(raw, np.int32, cells, o).reshape(height, width, 2); o += 4 * cells
        out.append({"pair": tuple(int(v) for v in lr), "fx": sc[0], "fy": sc[1], "cx": sc[2], "cy": sc[3],
                    "baseline": sc[4], "base_T_rect": base, "map_left": ml, "map_right": mr})
    assert o == len(raw)
    return out


def read_run(path: Path, n_frames: int, pairs: int) -> dict:
    """Output of ``rig_from_calib run``."""
    raw = Path(path).read_bytes()
    t_abs, stats, rig = [], [], []
    o = 0
    for _ in range(n_frames):
        t_abs.append(np.frombuffer(raw, np.float64, 16 * pairs, o).reshape(pairs, 4, 4)); o += 128 * pairs
        stats.append(np.frombuffer(raw, np.int32, 8 * pairs, o).reshape(pairs, 8)); o += 32 * pairs
        if pairs > 1:
            rig.append(np.frombuffer(raw, np.float64, 16, o).reshape(4, 4)); o += 128
    pose = {"T": np.frombuffer(raw, np.float64, 16, o).reshape(4, 4)}; o += 128
    pose["cov"] = np.frombuffer(raw, np.float64, 36, o).reshape(6, 6); o += 288
    pose["ts"] = float(np.frombuffer(raw, np.float64, 1, o)[0]); o += 8
    pose["state"] = int(np.frombuffer(raw, np.int32, 1, o)[0]); o += 4
    pose["conf"] = float(np.frombuffer(raw, np.float32, 1, o)[0]); o += 4
    assert o == len(raw)
    return {"T_abs": np.stack(t_abs), "stats": np.stack(stats), "rig_T_abs": np.stack(rig) if rig else None, "pose": pose}
