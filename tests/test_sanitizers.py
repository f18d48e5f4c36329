"""SURVEY.md §5 robustness: the library's host C++ — calibration / rectification tables
(tslam_calib.cpp), the IMU filter (tslam_imu.cpp) and the sharded frame-range arithmetic
(tslam_ranges.h) — built with AddressSanitizer + UndefinedBehaviorSanitizer (`make sanitize`:
tests/c/host_check.cpp links the host sources into an executable of its own, any report aborts)
and run on the inputs the product tests use; its outputs must equal the ctypes library's and the
Python product's byte for byte.  CPU only."""

from __future__ import annotations

import ctypes
import shutil
import subprocess
from pathlib import Path

import numpy as np
import pytest

import native_caller
from helpers import C3_SOURCES, make_source, rig_calibration
from thor_slam_amd import _lib
from thor_slam_amd.calib import extract_cameras, stereo_pairs, stereo_rectify
from thor_slam_amd.imu import ImuNoise
from thor_slam_amd.synthetic import DRB_TO_RDF, SyntheticStereoSource

ROOT = Path(__file__).resolve().parents[1]
CSRC = ROOT / "thor-slam_amd" / "csrc"
EXE = CSRC / "build-asan" / "host_check"
ENV = {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=1", "UBSAN_OPTIONS": "print_stacktrace=1:halt_on_error=1",
       "PATH": "/usr/bin:/bin"}


def _has_asan() -> bool:
    if shutil.which("g++") is None:
        return False
    probe = subprocess.run(["g++", "-fsanitize=address,undefined", "-x", "c++", "-", "-o", "/dev/null"],
                           input="int main(){return 0;}", capture_output=True, text=True)
    return probe.returncode == 0


pytestmark = pytest.mark.skipif(not _has_asan(), reason="g++ with libasan / libubsan not available")


@pytest.fixture(scope="module")
def exe():
    subprocess.run(["make", "-s", "-C", str(CSRC), "build-asan/host_check"], check=True)
    return EXE


def _run(exe, *args):
    out = subprocess.run([str(exe), *map(str, args)], capture_output=True, text=True, env=ENV)
    assert out.returncode == 0, f"host_check {args[0]}: rc {out.returncode}\n{out.stderr[-3000:]}"
    assert "runtime error" not in out.stderr and "AddressSanitizer" not in out.stderr, out.stderr[-3000:]
    return out


def test_sanitizer_target_ranges(exe):
    """`make sanitize` (the Makefile target) builds the executable and runs the exhaustive range check."""
    out = subprocess.run(["make", "-s", "-C", str(CSRC), "sanitize"], capture_output=True, text=True)
    assert out.returncode == 0, out.stderr[-3000:]
    assert "cases" in out.stdout


def test_sanitized_rectification_tables_match_calib(exe, tmp_path):
    """The C3 brackets rig (4 sources, rotated mounts) and a distorted pair: the sanitized host code
    writes exactly the tables calib.py builds (tests/test_native_calib.py's bar)."""
    from helpers import rig_scene

    for cams in (rig_scene(names=C3_SOURCES, n=1)["cams"],
                 extract_cameras(rig_calibration(make_source(distorted=True)), 2)):
        native_caller.write_calib(cams, tmp_path / "calib.txt")
        _run(exe, "maps", tmp_path / "calib.txt", tmp_path / "maps.bin")
        pairs = stereo_pairs(cams)
        got = native_caller.read_maps(tmp_path / "maps.bin", len(pairs), 640, 400)
        for (l, r), g in zip(pairs, got):
            py = stereo_rectify(cams[l], cams[r])
            assert g["pair"] == (l, r)
            np.testing.assert_array_equal(g["map_left"], py.map_left)
            np.testing.assert_array_equal(g["map_right"], py.map_right)
            assert (g["fx"], g["fy"], g["cx"], g["cy"]) == (py.fx, py.fy, py.cx, py.cy)


def _imu_script(accel: bool, seed: int = 0):
    """A 30-frame sequence of the synthetic IMU in batches of 1..5, some frames without a sample,
    some lost (status 1), noisy visual motions."""
    src = SyntheticStereoSource(seed=seed, imu=True, gyro_noise=1e-3, accel_noise=0.02, n_frames=40,
                                gyro_bias=[2e-3, -1e-3, 3e-3])
    rng = np.random.default_rng(seed)
    n, batches, i = 30, [], 1
    while i < n:
        b = int(rng.integers(1, 6))
        idx = list(range(i, min(n, i + b)))
        dt = np.array([np.nan if k % 9 == 4 else 1.0 / src.fps for k in idx])
        gy = np.stack([src.imu_sample(k)["gyroscope"] for k in idx]).astype(np.float64)
        ac = np.stack([src.imu_sample(k)["accelerometer"] for k in idx]).astype(np.float64)
        st = np.array([1 if k % 7 == 0 else 0 for k in idx], dtype=np.int32)
        tr = []
        for k in idx:
            t = np.linalg.inv(src.camera_pose(k, 0)) @ src.camera_pose(k - 1, 0)
            t[:3, 3] += rng.normal(0, 1e-3, 3)
            tr.append(t)
        cv = np.stack([np.diag([1e-6] * 3 + [1e-8] * 3)] * len(idx))
        batches.append((dt, gy, ac, st, np.stack(tr), cv))
        i += b
    return src, batches


def _write_script(path, accel, ri, noise, lever, a0, batches):
    parts = [np.array([int(accel), len(batches)], np.int32).tobytes(), ri.tobytes(), noise.tobytes(), lever.tobytes(),
             a0.tobytes()]
    for dt, gy, ac, st, tr, cv in batches:
        pad = np.zeros(len(st) & 1, np.int32)
        parts += [np.array([len(dt), 0], np.int32).tobytes(), dt.tobytes(), gy.tobytes(), ac.tobytes(), tr.tobytes(),
                  cv.tobytes(), st.tobytes(), pad.tobytes()]
    Path(path).write_bytes(b"".join(parts))


def _library_run(accel, ri, noise, lever, a0, batches) -> bytes:
    """The same calls through the shipped libtslam_hip.so (ctypes)."""
    lib = _lib.load_library()
    f = ctypes.c_void_p()
    dp = lambda a: None if a is None else np.ascontiguousarray(a).ctypes.data   # noqa: E731
    _lib._check(lib.tslam_imu_create(dp(ri), dp(noise), dp(lever), int(accel), ctypes.byref(f)))
    _lib._check(lib.tslam_imu_begin(f, dp(a0) if accel else None))
    out = []
    for dt, gy, ac, st, tr, cv in batches:
        n = len(dt)
        steps = (_lib.ImuStep * n)()
        valid = np.zeros(n, np.int32)
        _lib._check(lib.tslam_imu_batch_priors(f, n, dp(dt), dp(gy), dp(ac) if accel else None, steps, dp(valid)))
        _lib._check(lib.tslam_imu_absorb(f, n, dp(dt), dp(gy), dp(ac) if accel else None, dp(st), dp(tr), dp(cv)))
        s = _lib.ImuState()
        _lib._check(lib.tslam_imu_get_state(f, ctypes.byref(s)))
        out += [bytes(steps), valid.tobytes(), bytes(s)]
    lib.tslam_imu_destroy(f)
    return b"".join(out)


@pytest.mark.parametrize("accel", [True, False])
def test_sanitized_imu_filter_matches_library(exe, tmp_path, accel):
    """The IMU filter over a scripted sequence (ragged batches, missing samples, lost frames):
    every prior, validity flag and state the sanitized build writes equals the library's bytes."""
    src, batches = _imu_script(accel)
    n = ImuNoise()
    noise = np.array([n.gyro_density, n.gyro_random_walk, n.acc_density, n.acc_random_walk, n.rot_floor, n.trans_floor,
                      n.v0_sigma, n.ba0_sigma, n.bg0_sigma, n.vis_rot_floor], np.float64)
    ri = np.ascontiguousarray(DRB_TO_RDF[:3, :3], np.float64)
    lever = np.array([0.0375, 0.0, 0.0])
    a0 = np.asarray(src.imu_sample(0)["accelerometer"], np.float64)
    _write_script(tmp_path / "imu.bin", accel, ri, noise, lever, a0, batches)
    _run(exe, "imu", tmp_path / "imu.bin", tmp_path / "out.bin")
    assert (tmp_path / "out.bin").read_bytes() == _library_run(accel, ri, noise, lever, a0, batches)
