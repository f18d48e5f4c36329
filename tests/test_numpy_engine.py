"""The NumPy CPU SlamEngine (oracle/numpy_engine.py; BASELINE.json configs[0], SURVEY.md §7 step
2) through the reference's own loop (scripts/run_slam.py:299-328: a CameraRig, initialize with the
rig's calibration and no config, process_frames per synchronised set).  CPU only."""

from __future__ import annotations

from concurrent.futures import ProcessPoolExecutor

import numpy as np

from helpers import make_source, rel_frobenius
from oracle import numpy_slam as O
from oracle.numpy_engine import NumpySlamEngine
from thor_slam_amd.calib import extract_cameras, stereo_pairs, stereo_rectify
from thor_slam_amd.camera import CameraRig, Extrinsics
from thor_slam_amd.params import HipSlamConfig
from thor_slam_amd.slam.interface import SlamEngine, TrackingState
from thor_slam_amd.synthetic import CachedStereoSource


def _render(args):
    seed, idx = args
    src = make_source(seed, n_frames=200)
    return [src.render_stereo_sequence(1, start=i)[0] for i in idx]


def _frames(seed: int, n: int, workers: int = 8) -> np.ndarray:
    chunks = [list(range(n))[k::workers] for k in range(workers)]
    out = np.empty((n, 2, 400, 640), np.uint8)
    with ProcessPoolExecutor(max_workers=workers) as ex:
        for ch, frs in zip(chunks, ex.map(_render, [(seed, c) for c in chunks])):
            for i, f in zip(ch, frs):
                out[i] = f
    return out


def _tracker_run(args):
    """A standalone OracleTracker over the frames (the reference of the comparison)."""
    frames, rect = args
    trk = O.OracleTracker(HipSlamConfig(), rect)
    out = []
    for i in range(len(frames)):
        r = trk.step(frames[i, 0], frames[i, 1])
        out.append((int(r["status"]), r["world_T_cam"]))
    return out


def test_c1_through_the_reference_loop_matches_the_oracle_tracker():
    """Config C1: 100 synthetic 640x400 stereo frames, NumpySlamEngine built as run_slam.py:299-300
    builds the engine (no config: loop closure on, the rig's identity IMU idle), fed by CameraRig
    synchronised sets: every frame's tracked pose is the standalone OracleTracker's byte for byte,
    and the published SlamPose is its base_link conjugate."""
    n = 100
    frames = _frames(5, n)
    src = make_source(5, n_frames=200)
    cached = CachedStereoSource(frames, seed=5, n_frames=200)
    rig = CameraRig([cached], rig_extrinsics={cached.name: Extrinsics.from_4x4_matrix(cached.rig_T_source)})
    rig.start()
    cams = extract_cameras(rig.calibration, 2)
    (li, ri), = stereo_pairs(cams)
    r = stereo_rectify(cams[li], cams[ri])
    rect = dict(fx=r.fx, fy=r.fy, cx=r.cx, cy=r.cy, baseline=r.baseline, map_l=r.map_left, map_r=r.map_right)
    with ProcessPoolExecutor(max_workers=1) as ex:
        ref = ex.submit(_tracker_run, (frames, rect))
        eng = NumpySlamEngine(num_cameras=2)
        assert isinstance(eng, SlamEngine)
        eng.initialize(rig.calibration)
        assert eng._config.enable_loop_closure and eng._loop is not None
        poses = [eng.process_frames(rig.get_synchronized_frames()) for _ in range(n)]
        want = ref.result()
    bt = eng._E[0]
    tracked = 0
    for i, (p, (st, wTc)) in enumerate(zip(poses, want)):
        got = eng.results[i][0]
        assert int(got["status"]) == st, i
        np.testing.assert_array_equal(got["world_T_cam"], wTc, err_msg=f"frame {i}")
        if st == 1:
            assert p is None
            continue
        tracked += st == 0
        assert rel_frobenius(p.to_4x4_matrix(), bt @ wTc @ np.linalg.inv(bt)) < 1e-12, i
    assert tracked >= 90 and eng.get_tracking_state() == TrackingState.TRACKING
    # the body-frame motion agrees with the rendered ground truth (FLU base_link)
    gt = np.linalg.inv(src.ground_truth_body(0)) @ src.ground_truth_body(n - 1)
    assert np.linalg.norm(poses[-1].position - gt[:3, 3]) < 0.1 * np.linalg.norm(gt[:3, 3]) + 5e-3
    assert not eng._loop.loops and len(eng._loop.frames) >= 18   # keyframes every 5 frames, no loop in 100
    eng.shutdown()


def test_imu_lagged_priors_match_run_sequence():
    """With an IMU on the rig the engine's lagged priors (imu_prior_lag = 1, batch 1) equal
    oracle/numpy_imu.run_sequence(batch=1, lag=1) on the same frames and samples."""
    from oracle import numpy_imu as OI
    from thor_slam_amd.camera.types import IMUExtrinsics
    from thor_slam_amd.synthetic import DRB_TO_RDF, SyntheticStereoSource

    n = 6
    src = SyntheticStereoSource(seed=0, imu=True, gyro_noise=1e-4, accel_noise=0.01, n_frames=40)
    rig_T = src.rig_T_source
    rig = CameraRig([src], rig_extrinsics={src.name: Extrinsics.from_4x4_matrix(rig_T)}, imu_source=src.name,
                    imu_extrinsics=IMUExtrinsics(src.name, Extrinsics.from_4x4_matrix(rig_T @ DRB_TO_RDF)))
    rig.start()
    cfg = HipSlamConfig(imu_fusion=True, imu_accel=True, enable_loop_closure=False)
    eng = NumpySlamEngine(num_cameras=2, config=cfg)
    eng.initialize(rig.calibration)
    sets = [rig.get_synchronized_frames() for _ in range(n)]
    for s in sets:
        eng.process_frames(s)
    frames = np.stack([np.stack([s.frame_sets[src.name].frames[c].image for c in (0, 1)]) for s in sets])
    samples = []
    for i in range(n):
        sm = src.imu_sample(i)
        samples.append((None if i == 0 else src.timestamp(i) - src.timestamp(i - 1), sm["gyroscope"], sm["accelerometer"]))
    cams = extract_cameras(rig.calibration, 2)
    (li, ri), = stereo_pairs(cams)
    r = stereo_rectify(cams[li], cams[ri])
    bt = cams[li].extrinsics.to_4x4_matrix() @ r.left_optical_T_rect()
    rect_T_imu = np.linalg.inv(bt) @ rig.calibration.imu_extrinsics.to_4x4_matrix()
    filt = OI.ImuFilter(rect_T_imu[:3, :3], cfg.accelerometer_noise_density, cfg.accelerometer_random_walk,
                        cfg.gyroscope_noise_density, cfg.gyroscope_random_walk, cfg.imu_rot_floor, cfg.imu_trans_floor,
                        ba0_sigma=cfg.imu_accel_bias_sigma, bg0_sigma=cfg.imu_gyro_bias_sigma, lever=rect_T_imu[:3, 3],
                        accel=True, vis_rot_floor=cfg.imu_vis_rot_floor)
    trk = O.OracleTracker(cfg, dict(fx=r.fx, fy=r.fy, cx=r.cx, cy=r.cy, baseline=r.baseline, map_l=r.map_left,
                                    map_r=r.map_right))
    want = OI.run_sequence(trk, frames, samples, 1, filt, lag=cfg.imu_prior_lag)
    for i in range(n):
        got = eng.results[i][0]
        assert int(got["status"]) == int(want[i]["status"]), i
        np.testing.assert_array_equal(got["world_T_cam"], want[i]["world_T_cam"], err_msg=f"frame {i}")
    assert eng._filt is not None and eng._filt.ready
    eng.shutdown()
