"""A native (gcc-built C) caller creates its handle from raw calibration with tslam_create_rig and
drives it through the asynchronous host boundary (tslam_submit_host / tslam_poll_batch /
tslam_poll_pose): its poses must be the bytes Python gets from the same entry points over ctypes
(Handle.from_cameras), and the poses of the handle HipSlamEngine builds through
thor_slam_amd/calib.py (Python rectification, set_rig for multi-pair rigs) up to the last bits of
the rectified intrinsics (tables byte-identical, tests/test_native_calib.py; baseline within
1e-14 m, so poses within 1e-12)."""

import subprocess

import numpy as np
import pytest

import native_caller
from helpers import make_source, rig_calibration, rig_scene
from thor_slam_amd._lib import Handle, make_params
from thor_slam_amd.calib import extract_cameras, stereo_pairs, stereo_rectify
from thor_slam_amd.params import HipSlamConfig

pytestmark = pytest.mark.gpu


def _python_path(cams, frames, cfg, batch, native: bool):
    pairs = stereo_pairs(cams)
    if native:
        h = Handle.from_cameras(cams, cfg, max_batch=batch)
    else:
        rects = [stereo_rectify(cams[l], cams[r]) for l, r in pairs]
        h = Handle(rects, cfg, max_batch=batch)
        if len(pairs) > 1:
            h.set_rig([cams[l].extrinsics.to_4x4_matrix() @ r.left_optical_T_rect() for (l, _), r in zip(pairs, rects)])
    t_abs, stats, rig = [], [], []
    for f0 in range(0, len(frames), batch):
        nb = min(batch, len(frames) - f0)
        h.submit_host(np.ascontiguousarray(frames[f0:f0 + nb]), [0.05 * (f0 + i) for i in range(nb)])
        res = h.poll_batch(block=True)
        assert res["first_frame"] == f0 and res["n"] == nb
        t_abs.append(res["T_abs"])
        stats.append(res["stats"])
        rig.append(res["rig"]["T_abs"])
    pose = h.poll_pose()
    h.close()
    return np.concatenate(t_abs), np.concatenate(stats), np.concatenate(rig), pose


@pytest.mark.parametrize("case", ["rig2", "distorted"])
def test_c_caller_create_rig_matches_python_handle(case, tmp_path):
    cfg = HipSlamConfig()
    if case == "rig2":
        sc = rig_scene(n=8)
        cams, frames, batch = sc["cams"], sc["frames"], 4
    else:
        src = make_source(distorted=True)
        cams = extract_cameras(rig_calibration(src), 2)
        frames, batch = src.render_stereo_sequence(6), 3
    n, n_pairs = len(frames), len(stereo_pairs(cams))
    exe = native_caller.build()
    native_caller.write_calib(cams, tmp_path / "calib.txt")
    (tmp_path / "params.bin").write_bytes(bytes(make_params(cfg, batch, 0)))
    (tmp_path / "frames.bin").write_bytes(np.ascontiguousarray(frames, dtype=np.uint8).tobytes())
    subprocess.run([str(exe), "run", str(tmp_path / "calib.txt"), str(tmp_path / "params.bin"), str(tmp_path / "frames.bin"),
                    str(n), str(batch), str(tmp_path / "out.bin")], check=True, timeout=90)
    got = native_caller.read_run(tmp_path / "out.bin", n, n_pairs)

    t_abs, stats, rig, pose = _python_path(cams, frames, cfg, batch, native=True)
    assert (stats[:, :, 0] == 0).sum() >= n_pairs * (n - 2)   # tracked, not a vacuous comparison
    np.testing.assert_array_equal(got["stats"], stats)
    np.testing.assert_array_equal(got["T_abs"], t_abs)
    if n_pairs > 1:
        np.testing.assert_array_equal(got["rig_T_abs"], rig)
    assert got["pose"]["ts"] == pytest.approx(0.05 * (n - 1)) == pose["timestamp"]
    assert got["pose"]["state"] == pose["state"]
    np.testing.assert_array_equal(got["pose"]["T"], pose["T"])

    t_py, stats_py, rig_py, _ = _python_path(cams, frames, cfg, batch, native=False)
    # same tables: same matches, same RANSAC winners (stats[6..7] hold sigma^2, a float of the solve)
    np.testing.assert_array_equal(got["stats"][..., :6], stats_py[..., :6])
    np.testing.assert_allclose(got["T_abs"], t_py, rtol=0, atol=1e-12)
    if n_pairs > 1:
        np.testing.assert_allclose(got["rig_T_abs"], rig_py, rtol=0, atol=1e-12)
