"""The C-ABI library loads and exports every symbol include/tslam.h declares; the ctypes
mirrors match the C struct layouts; argument validation fails cleanly (no GPU needed)."""

import ctypes
import re
import subprocess
from pathlib import Path

import pytest

from thor_slam_amd import _lib

ROOT = Path(__file__).resolve().parents[1]
HEADER = ROOT / "include" / "tslam.h"


def declared_functions() -> set[str]:
    text = HEADER.read_text()
    return set(re.findall(r"^\s*(?:const\s+)?[a-z0-9_]+\s*\*?\s*(tslam_[a-z_]+)\s*\(", text, re.M))


def test_header_declarations_match_bindings():
    assert declared_functions() == set(_lib.exported_symbols())


def test_library_exports_every_symbol():
    lib = _lib.load_library()
    for name in declared_functions():
        assert hasattr(lib, name), name
    assert lib.tslam_abi_version() == int(re.search(r"#define TSLAM_ABI_VERSION (\d+)", HEADER.read_text()).group(1))
    out = subprocess.run(["nm", "-D", "--defined-only", str(_lib.LIB_PATH)], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r" T (tslam_[a-z_]+)", out))
    assert declared_functions() <= exported


def test_struct_layouts_match_c(tmp_path):
    src = tmp_path / "probe.c"
    src.write_text(f"""
#include <stdio.h>
#include <stddef.h>
#include "{HEADER}"
int main(void) {{
  printf("%zu %zu %zu %zu %zu %zu %zu %zu %zu %zu\\n", sizeof(tslam_params), offsetof(tslam_params, ransac_thr_px),
         offsetof(tslam_params, ransac_seed), offsetof(tslam_params, ransac_splits),
         offsetof(tslam_params, ba_window), offsetof(tslam_params, ba_lambda), offsetof(tslam_params, rgbd),
         offsetof(tslam_params, refine_block), sizeof(tslam_stereo_desc), offsetof(tslam_stereo_desc, map_left));
  return 0;
}}""")
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-std=c99", str(src), "-o", str(exe)], check=True)
    got = list(map(int, subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()))
    P, S = _lib.Params, _lib.StereoDesc
    assert got == [ctypes.sizeof(P), P.ransac_thr_px.offset, P.ransac_seed.offset, P.ransac_splits.offset,
                   P.ba_window.offset, P.ba_lambda.offset, P.rgbd.offset, P.refine_block.offset, ctypes.sizeof(S),
                   S.map_left.offset]


def test_invalid_arguments_fail_cleanly():
    from thor_slam_amd.params import HipSlamConfig

    lib = _lib.load_library()
    desc = _lib.StereoDesc(640, 400, 384.0, 384.0, 319.5, 199.5, 0.075, None, None)
    h = ctypes.c_void_p()
    bad = [
        dict(n_pairs=0), dict(max_batch=0), dict(ransac_splits=99), dict(refine_block=64),
    ]
    for kw in bad:
        prm = _lib.make_params(HipSlamConfig(), kw.get("max_batch", 4), kw.get("n_pairs", 1), kw.get("ransac_splits", 0),
                               refine_block=kw.get("refine_block", 0))
        rc = lib.tslam_create(ctypes.byref(desc), ctypes.byref(prm), 0, ctypes.byref(h))
        assert rc == -1, kw
        assert lib.tslam_last_error()
    prm = _lib.make_params(HipSlamConfig(n_levels=6), 4, 1)  # coarsest level too small for the margin
    assert lib.tslam_create(ctypes.byref(desc), ctypes.byref(prm), 0, ctypes.byref(h)) == -1
    assert b"coarsest" in lib.tslam_last_error()
    assert lib.tslam_submit(None, None, 1, None) == -1
    assert lib.tslam_destroy(None) == 0


def test_missing_library_raises(tmp_path):
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        _lib.load_library(tmp_path / "nope.so")
