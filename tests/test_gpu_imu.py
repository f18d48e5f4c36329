"""IMU fusion: a gyro-predicted rotation prior in A7's Gauss-Newton.

HIP (``tslam_set_motion_prior`` + ``k_refine``) vs the oracle's ``refine(prior=...)`` on the
same frames and priors: RANSAC winners identical (the prior does not touch RANSAC), poses within
1e-9 relative Frobenius.  Then the engine with a synthetic IMU source end to end."""

from __future__ import annotations

import numpy as np
import pytest
from scipy.spatial.transform import Rotation

from helpers import make_source, rel_frobenius, scenario
from oracle import numpy_slam as O

pytestmark = pytest.mark.gpu


def _priors(sc, n, err=1e-3, weight=2e5):
    """Relative rectified-left rotations from the renderer, off by a fixed 1 mrad rotation."""
    src, rect = sc["src"], sc["rect"]
    bad = Rotation.from_rotvec([err, -err, 0.5 * err]).as_matrix()
    rot = np.tile(np.eye(3), (n, 1, 1))
    w = np.zeros(n)
    for g in range(1, n):
        r0 = src.camera_pose(g - 1, 0)[:3, :3] @ rect.rect_left.T
        r1 = src.camera_pose(g, 0)[:3, :3] @ rect.rect_left.T
        rot[g] = bad @ (r1.T @ r0)
        w[g] = weight
    return rot, w


def test_motion_prior_matches_oracle():
    import torch

    from thor_slam_amd._lib import Handle

    n = 4
    sc = scenario(seed=0, n=n)
    cfg, rect = sc["cfg"], sc["rect"]
    rot, w = _priors(sc, n)
    trk = O.OracleTracker(cfg, dict(fx=rect.fx, fy=rect.fy, cx=rect.cx, cy=rect.cy, baseline=rect.baseline,
                                    map_l=rect.map_left, map_r=rect.map_right))
    want = [trk.step(sc["frames"][g, 0], sc["frames"][g, 1], prior=(rot[g], w[g])) for g in range(n)]
    h = Handle([rect], cfg, max_batch=n)
    h.set_motion_prior(rot[:, None], w[:, None])
    dev = torch.from_numpy(np.ascontiguousarray(sc["frames"])).cuda()
    h.submit(dev.data_ptr(), n, torch.cuda.current_stream().cuda_stream)
    res = h.read_poses(n)
    h.close()
    for g in range(1, n):
        st = res["stats"][g, 0]
        assert st[0] == want[g]["status"] == 0 and st[4] == want[g]["best_hyp"] and st[2] == want[g]["n_inliers"]
        assert rel_frobenius(res["T_rel"][g, 0], want[g]["T"]) < 1e-9
        assert rel_frobenius(res["cov"][g, 0], want[g]["cov"]) < 1e-6
        # the prior pulled the rotation away from the vision-only solution, towards the prior
        vis = sc["oracle"][g]["T"][:3, :3]
        d_prior = np.linalg.norm(Rotation.from_matrix(res["T_rel"][g, 0][:3, :3] @ rot[g].T).as_rotvec())
        d_vis = np.linalg.norm(Rotation.from_matrix(vis @ rot[g].T).as_rotvec())
        assert d_prior < d_vis


def test_engine_with_imu_source():
    from thor_slam_amd.camera import CameraRig, Extrinsics
    from thor_slam_amd.camera.types import IMUExtrinsics
    from thor_slam_amd.params import HipSlamConfig
    from thor_slam_amd.slam.hip_engine import HipSlamEngine
    from thor_slam_amd.synthetic import DRB_TO_RDF, SyntheticStereoSource

    def run(fusion):
        src = SyntheticStereoSource(seed=0, imu=True, gyro_noise=1e-3)
        rig_T = src.rig_T_source
        rig = CameraRig([src], rig_extrinsics={src.name: Extrinsics.from_4x4_matrix(rig_T)}, imu_source=src.name,
                        imu_extrinsics=IMUExtrinsics(src.name, Extrinsics.from_4x4_matrix(rig_T @ DRB_TO_RDF)))
        rig.start()
        eng = HipSlamEngine(num_cameras=2, config=HipSlamConfig(imu_fusion=fusion, batch_size=3))
        eng.initialize(rig.calibration)
        for _ in range(9):
            fs = rig.get_synchronized_frames()
            assert fs.sensor_data is not None
            eng.process_frames(fs)
        eng.flush()
        pose = eng._latest_pose
        eng.shutdown()
        gt = np.linalg.inv(src.ground_truth_body(0)) @ src.ground_truth_body(8)
        return pose, gt

    p_imu, gt = run(True)
    p_vis, _ = run(False)
    e_imu = np.linalg.norm(p_imu.position - gt[:3, 3])
    e_vis = np.linalg.norm(p_vis.position - gt[:3, 3])
    assert e_imu < 0.1 * np.linalg.norm(gt[:3, 3]) + 2e-3
    r_imu = np.linalg.norm(Rotation.from_matrix(p_imu.to_4x4_matrix()[:3, :3].T @ gt[:3, :3]).as_rotvec())
    r_vis = np.linalg.norm(Rotation.from_matrix(p_vis.to_4x4_matrix()[:3, :3].T @ gt[:3, :3]).as_rotvec())
    assert r_imu < r_vis + 2e-3 and e_imu < e_vis + 5e-3


def oracle_filter(cfg, rect_T_imu, accel=True):
    from oracle import numpy_imu as OI

    return OI.ImuFilter(rect_T_imu[:3, :3], cfg.accelerometer_noise_density, cfg.accelerometer_random_walk,
                        cfg.gyroscope_noise_density, cfg.gyroscope_random_walk, cfg.imu_rot_floor, cfg.imu_trans_floor,
                        ba0_sigma=cfg.imu_accel_bias_sigma, bg0_sigma=cfg.imu_gyro_bias_sigma, lever=rect_T_imu[:3, 3],
                        accel=accel, vis_rot_floor=cfg.imu_vis_rot_floor)


def _imu_rig(n_frames=40, blackout=None, accel_noise=0.0, gyro_noise=0.0, gyro_bias=None):
    from thor_slam_amd.camera import CameraRig, Extrinsics
    from thor_slam_amd.camera.types import IMUExtrinsics
    from thor_slam_amd.synthetic import DRB_TO_RDF, SyntheticStereoSource

    src = SyntheticStereoSource(seed=0, imu=True, gyro_noise=gyro_noise, accel_noise=accel_noise, blackout=blackout,
                                n_frames=n_frames, gyro_bias=gyro_bias)
    rig_T = src.rig_T_source
    rig = CameraRig([src], rig_extrinsics={src.name: Extrinsics.from_4x4_matrix(rig_T)}, imu_source=src.name,
                    imu_extrinsics=IMUExtrinsics(src.name, Extrinsics.from_4x4_matrix(rig_T @ DRB_TO_RDF)))
    return src, rig


def _run_engine(rig, n, cfg, num_cameras=2, keep=None):
    from thor_slam_amd.slam.hip_engine import HipSlamEngine

    rig.start()
    eng = HipSlamEngine(num_cameras=num_cameras, config=cfg)
    eng.initialize(rig.calibration)
    got = []
    orig = eng._publish

    def record(res, stamps, g0):
        rec = {k: np.array(res[k][:len(stamps)]) for k in ("T_abs", "T_rel", "stats")}
        if "rig" in res:
            rec.update({"rig_" + k: np.array(res["rig"][k][:len(stamps)]) for k in ("T_abs", "stats")})
        got.append(rec)
        orig(res, stamps, g0)

    eng._publish = record
    for _ in range(n):
        eng.process_frames(rig.get_synchronized_frames())
    eng.flush()
    rects = eng._rects
    if keep is not None:
        keep["imu"] = eng._imu
        keep["pose"] = eng._latest_pose
    eng.shutdown()
    cat = {k: np.concatenate([g[k] for g in got]) for k in got[0]}
    return cat, rects


@pytest.mark.parametrize("batch,lag", [(4, 1), (1, 1), (4, 0)])
def test_accelerometer_prior_and_dropout_match_oracle(batch, lag):
    """The engine's gyro + accelerometer leg (host filter -> tslam_set_motion_prior -> k_refine's
    translation prior and k_chain's IMU chaining) against oracle/numpy_imu.run_sequence on the same
    frames and samples, across a 3-frame visual dropout: statuses and RANSAC winners identical,
    T_abs within 1e-9.  With imu_prior_lag 1 (the default) the prior of batch s lacks the vision of
    batch s - 1 (lagged_priors), so batches stay in flight; batch 1 is the default drop-in path."""
    from oracle import numpy_imu as OI
    from thor_slam_amd.params import HipSlamConfig

    n = 20
    src, rig = _imu_rig(blackout=(9, 12), accel_noise=0.01, gyro_noise=1e-4)
    cfg = HipSlamConfig(imu_fusion=True, imu_accel=True, batch_size=batch, imu_prior_lag=lag)
    res, rects = _run_engine(rig, n, cfg)
    rect = rects[0]
    cal = rig.calibration
    from thor_slam_amd.calib import extract_cameras

    cams = extract_cameras(cal, 2)
    bt = cams[0].extrinsics.to_4x4_matrix() @ rect.left_optical_T_rect()
    rect_T_imu = np.linalg.inv(bt) @ cal.imu_extrinsics.to_4x4_matrix()
    samples = []
    for i in range(n):
        s = src.imu_sample(i)
        dt = None if i == 0 else src.timestamp(i) - src.timestamp(i - 1)
        samples.append((dt, s["gyroscope"], s["accelerometer"]))
    trk = O.OracleTracker(cfg, dict(fx=rect.fx, fy=rect.fy, cx=rect.cx, cy=rect.cy, baseline=rect.baseline,
                                    map_l=rect.map_left, map_r=rect.map_right))
    frames = np.stack([np.stack([src.render_image(i, 0), src.render_image(i, 1)]) for i in range(n)])
    filt = oracle_filter(cfg, rect_T_imu)
    want = OI.run_sequence(trk, frames, samples, batch, filt, lag=cfg.imu_prior_lag)
    status = [int(w["status"]) for w in want]
    assert status[9:13] == [1, 1, 1, 1] and status[13:] == [0] * (n - 13)   # the dropout, then tracking
    for g in range(n):
        st = res["stats"][g, 0]
        assert st[0] == want[g]["status"], g
        if want[g]["status"] == 0:
            assert st[4] == want[g]["best_hyp"] and st[2] == want[g]["n_inliers"], g
        assert rel_frobenius(res["T_abs"][g, 0], want[g]["world_T_cam"]) < 1e-9, g


def test_accelerometer_bridges_a_visual_dropout():
    """Through a 6-frame dropout the gyro-only prior cannot move the camera; the accelerometer
    leg carries it, so the end-of-sequence position error drops well below the gyro-only one."""
    from thor_slam_amd.params import HipSlamConfig

    n = 30
    errs = {}
    for accel in (False, True):
        src, rig = _imu_rig(blackout=(10, 16), accel_noise=0.01, gyro_noise=1e-4)
        cfg = HipSlamConfig(imu_fusion=True, imu_accel=accel, batch_size=1)
        res, rects = _run_engine(rig, n, cfg)
        rect = rects[0]
        cams_T = [src.camera_pose(i, 0) for i in (0, n - 1)]
        # ground truth in the rectified-left frame of frame 0 (rectification is the identity here)
        gt = np.linalg.inv(cams_T[0]) @ cams_T[1]
        assert rect.is_identity and int(res["stats"][n - 1, 0, 0]) == 0
        errs[accel] = np.linalg.norm(res["T_abs"][n - 1, 0][:3, 3] - gt[:3, 3])
    travelled = 0.5 * 7 / 30.0   # 0.5 m/s through the 7 untracked frames
    assert errs[False] > 0.5 * travelled
    assert errs[True] < 0.25 * errs[False], errs


def test_gyro_bias_estimated_and_drift_reduced():
    """A constant gyroscope bias (30, -20, 25 mrad/s, an uncalibrated MEMS gyro): with the bias
    state (learnt from the vision-only motions behind the prior-weighted solutions) the estimate
    comes within 25 % of it and the trajectory through a 6-frame visual dropout ends closer to the
    truth than with the bias pinned at zero (imu_gyro_bias_sigma ~ 0: no bias state, as round 2's
    filter).  The residual estimate error is the vision's own correlated rotation error (~5 mrad/s
    of yaw on this sequence), which no loosely coupled filter can tell from a bias."""
    from thor_slam_amd.params import HipSlamConfig

    bias = np.array([0.03, -0.02, 0.025])
    n = 60
    out = {}
    for sigma in (0.01, 1e-9):
        src, rig = _imu_rig(n_frames=n, blackout=(40, 46), accel_noise=0.01, gyro_noise=1e-4, gyro_bias=bias)
        cfg = HipSlamConfig(batch_size=4, imu_gyro_bias_sigma=sigma, enable_loop_closure=False)
        keep = {}
        res, rects = _run_engine(rig, n, cfg, keep=keep)
        gt = np.linalg.inv(src.camera_pose(0, 0)) @ src.camera_pose(n - 1, 0)
        T = res["T_abs"][n - 1, 0]
        out[sigma] = {"bg": keep["imu"].st.bg.copy(), "t": np.linalg.norm(T[:3, 3] - gt[:3, 3]),
                      "r": Rotation.from_matrix(T[:3, :3].T @ gt[:3, :3]).magnitude(),
                      "status": res["stats"][:, 0, 0]}
    est = out[0.01]
    assert (est["status"][40:46] == 1).all() and est["status"][-1] == 0
    assert np.linalg.norm(est["bg"] - bias) < 0.25 * np.linalg.norm(bias), est["bg"]
    assert np.linalg.norm(out[1e-9]["bg"]) < 1e-6
    assert est["r"] < 0.5 * out[1e-9]["r"], (est["r"], out[1e-9]["r"])
    assert est["t"] < out[1e-9]["t"], (est["t"], out[1e-9]["t"])


def test_rig_imu_dropout_matches_oracle():
    """A two-source rig with the IMU on source 0 and every camera blind for frames 9-11: the
    engine (pair priors moved through the rig, k_rig_prior's body prediction in the rig chain,
    the filter absorbing the rig's motion) against oracle/numpy_imu.run_rig_sequence: rig
    statuses identical, rig world_T_base within 1e-9 through and after the dropout."""
    import json
    from pathlib import Path

    from oracle import numpy_imu as OI
    from thor_slam_amd.calib import extract_cameras, stereo_pairs, stereo_rectify
    from thor_slam_amd.camera import CameraRig, Extrinsics
    from thor_slam_amd.camera.types import IMUExtrinsics
    from thor_slam_amd.params import HipSlamConfig
    from thor_slam_amd.synthetic import DRB_TO_RDF, RoomScene, SyntheticStereoSource, circle_trajectory

    n, batch = 16, 4
    names = ("192.168.2.21", "192.168.2.25")
    mats = json.loads((Path(__file__).parent / "golden" / "brackets_joints.json").read_text())
    scene, traj = RoomScene(seed=0), circle_trajectory(40)
    srcs = [SyntheticStereoSource(name=nm, scene=scene, trajectory=traj, rig_T_source=np.array(mats[nm]), seed=k,
                                  imu=(k == 0), accel_noise=0.01, gyro_noise=1e-4, blackout=(9, 12))
            for k, nm in enumerate(names)]
    base_T_imu = np.array(mats[names[0]]) @ DRB_TO_RDF
    rig = CameraRig(srcs, rig_extrinsics={nm: Extrinsics.from_4x4_matrix(np.array(mats[nm])) for nm in names},
                    imu_source=names[0], imu_extrinsics=IMUExtrinsics(names[0], Extrinsics.from_4x4_matrix(base_T_imu)))
    cfg = HipSlamConfig(batch_size=batch, enable_loop_closure=False)
    res, rects = _run_engine(rig, n, cfg, num_cameras=4)
    cams = extract_cameras(rig.calibration, 4)
    pairs = stereo_pairs(cams)
    E = [cams[l].extrinsics.to_4x4_matrix() @ r.left_optical_T_rect() for (l, _), r in zip(pairs, rects)]
    by = {s.name: s for s in srcs}
    frames = np.stack([np.stack([by[cams[l].source_name].render_image(i, c) for l, _ in pairs for c in (0, 1)])
                       for i in range(n)])
    samples = []
    for i in range(n):
        sm = srcs[0].imu_sample(i)
        dt = None if i == 0 else srcs[0].timestamp(i) - srcs[0].timestamp(i - 1)
        samples.append((dt, sm["gyroscope"], sm["accelerometer"]))
    trks = [O.OracleTracker(cfg, dict(fx=r.fx, fy=r.fy, cx=r.cx, cy=r.cy, baseline=r.baseline, map_l=r.map_left,
                                      map_r=r.map_right)) for r in rects]
    filt = oracle_filter(cfg, np.linalg.inv(E[0]) @ base_T_imu)
    want = OI.run_rig_sequence(trks, frames, samples, batch, filt, E, cfg, lag=cfg.imu_prior_lag)
    status = [w["status"] for w in want]
    assert status[9:13] == [1] * 4 and status[13:] == [0] * (n - 13)   # frame 12 has no frame 11 to match
    for g in range(n):
        assert res["rig_stats"][g, 0] == want[g]["status"], g
        assert rel_frobenius(res["rig_T_abs"][g], want[g]["T_abs"]) < 1e-9, g


def test_engine_ba_imu_rotation_factors():
    """IMU fusion with local BA on one stereo pair: the gyro rotations of each keyframe interval,
    composed on the host, become the window's IMU rotation factors (tslam_ba_imu_factor) — one per
    keyframe after the first — and the BA keyframe orientations stay on the ground truth (no worse
    than the vision-only window by more than 0.5 mrad)."""
    from scipy.spatial.transform import Rotation

    from thor_slam_amd.camera import CameraRig, Extrinsics
    from thor_slam_amd.camera.types import IMUExtrinsics
    from thor_slam_amd.params import HipSlamConfig
    from thor_slam_amd.slam.hip_engine import HipSlamEngine
    from thor_slam_amd.synthetic import DRB_TO_RDF, SyntheticStereoSource

    def run(factors: bool):
        src = SyntheticStereoSource(seed=0, imu=True, gyro_noise=1e-3)
        rig_T = src.rig_T_source
        rig = CameraRig([src], rig_extrinsics={src.name: Extrinsics.from_4x4_matrix(rig_T)}, imu_source=src.name,
                        imu_extrinsics=IMUExtrinsics(src.name, Extrinsics.from_4x4_matrix(rig_T @ DRB_TO_RDF)))
        rig.start()
        # the separate rotation factors are the gyro-only path: with the accelerometer leg's inertial
        # factors on (the default) their records carry the gyro rotation rows instead
        eng = HipSlamEngine(num_cameras=2, config=HipSlamConfig(batch_size=4, ba_window=4, ba_kf_interval=2,
                                                                ba_iters=3, enable_loop_closure=False,
                                                                ba_inertial=False))
        eng.initialize(rig.calibration)
        calls = []
        inner = eng._handle.ba_imu_factor
        eng._handle.ba_imu_factor = lambda g, M, w, pair=0: (calls.append(g), inner(g, M, w, pair) if factors else None)
        for _ in range(16):
            eng.process_frames(rig.get_synchronized_frames())
        eng.flush()
        smap = eng.get_map()
        eng.shutdown()
        gt0 = src.ground_truth_body(0)
        rot_err = []
        for kf in smap.keyframe_poses:   # keyframe k by its timestamp
            k = min(range(16), key=lambda i: abs(src.timestamp(i) - kf.timestamp))
            gt = np.linalg.inv(gt0) @ src.ground_truth_body(k)
            rot_err.append(np.linalg.norm(Rotation.from_matrix(kf.to_4x4_matrix()[:3, :3].T @ gt[:3, :3]).as_rotvec()))
        return calls, rot_err

    calls, err_on = run(True)
    assert calls == [2, 4, 6, 8, 10, 12, 14], calls   # every keyframe after the first (interval 2)
    _, err_off = run(False)
    assert len(err_on) == len(err_off) == 8
    assert max(err_on) < max(err_off) + 5e-4, (err_on, err_off)


def test_engine_ba_inertial_factors():
    """IMU fusion (accelerometer leg) with local BA on one stereo pair: each keyframe interval's
    samples are preintegrated on the host (tslam_imu_preintegrate) and enter the window as
    tightly coupled inertial factors (tslam_ba_inertial_factor) — one per keyframe after the
    first; the window's velocities follow the camera's true velocity and the keyframe positions
    stay on the ground truth (no worse than without the factors by more than 5 mm)."""
    from thor_slam_amd.camera import CameraRig, Extrinsics
    from thor_slam_amd.camera.types import IMUExtrinsics
    from thor_slam_amd.params import HipSlamConfig
    from thor_slam_amd.slam.hip_engine import HipSlamEngine
    from thor_slam_amd.synthetic import DRB_TO_RDF, SyntheticStereoSource

    def run(inertial: bool):
        src = SyntheticStereoSource(seed=0, imu=True)
        rig_T = src.rig_T_source
        rig = CameraRig([src], rig_extrinsics={src.name: Extrinsics.from_4x4_matrix(rig_T)}, imu_source=src.name,
                        imu_extrinsics=IMUExtrinsics(src.name, Extrinsics.from_4x4_matrix(rig_T @ DRB_TO_RDF)))
        rig.start()
        eng = HipSlamEngine(num_cameras=2, config=HipSlamConfig(batch_size=4, ba_window=4, ba_kf_interval=2, ba_iters=3,
                                                                enable_loop_closure=False, ba_inertial=inertial))
        eng.initialize(rig.calibration)
        calls = []
        inner = eng._handle.ba_inertial_factor
        eng._handle.ba_inertial_factor = lambda g, rec, v0, pair=0: (calls.append(g), inner(g, rec, v0, pair))
        for _ in range(16):
            eng.process_frames(rig.get_synchronized_frames())
        eng.flush()
        smap = eng.get_map()
        ine = eng._handle.ba_read_inertial(0)
        frames = eng._handle.ba_read(0)["frames"]
        rects = eng._rects
        eng.shutdown()
        gt0 = src.ground_truth_body(0)
        pos_err = []
        for kf in smap.keyframe_poses:
            k = min(range(16), key=lambda i: abs(src.timestamp(i) - kf.timestamp))
            gt = np.linalg.inv(gt0) @ src.ground_truth_body(k)
            pos_err.append(np.linalg.norm(kf.to_4x4_matrix()[:3, 3] - gt[:3, 3]))
        return calls, pos_err, ine, frames, src

    calls, err_on, ine, frames, src = run(True)
    assert calls == [2, 4, 6, 8, 10, 12, 14], calls
    assert np.isfinite(ine["vel"]).all() and np.isfinite(ine["bias"]).all()
    # the camera's true speed at the window's keyframes (central differences of the left camera)
    c0 = src.camera_pose(0, 0)
    dt = 1.0 / src.fps
    for s, g in enumerate(frames):
        if g <= 0:
            continue
        p = [(np.linalg.inv(c0) @ src.camera_pose(int(g) + d, 0))[:3, 3] for d in (-1, 1)]
        v_true = (p[1] - p[0]) / (2 * dt)
        assert abs(np.linalg.norm(ine["vel"][s]) - np.linalg.norm(v_true)) < 0.05, (g, ine["vel"][s], v_true)
    calls_off, err_off, _, _, _ = run(False)
    assert calls_off == []
    assert len(err_on) == len(err_off) == 8
    assert max(err_on) < max(err_off) + 5e-3, (err_on, err_off)


def test_engine_rig_ba_inertial_factors():
    """A two-source rig with the IMU on source 0 and local BA (the rig's body window): the host
    preintegrates each keyframe interval in the body frame (tslam_imu_preintegrate with base_R_imu
    and the IMU's body position) and hands the body window its inertial factors (pair = n_pairs);
    the body velocities follow the rig's true speed and the keyframe positions stay on the ground
    truth (no worse than without the factors by more than 5 mm)."""
    import json
    from pathlib import Path

    from thor_slam_amd.camera import CameraRig, Extrinsics
    from thor_slam_amd.camera.types import IMUExtrinsics
    from thor_slam_amd.params import HipSlamConfig
    from thor_slam_amd.slam.hip_engine import HipSlamEngine
    from thor_slam_amd.synthetic import DRB_TO_RDF, RoomScene, SyntheticStereoSource, circle_trajectory

    n = 16
    names = ("192.168.2.21", "192.168.2.25")
    mats = json.loads((Path(__file__).parent / "golden" / "brackets_joints.json").read_text())

    def run(inertial: bool):
        scene, traj = RoomScene(seed=0), circle_trajectory(40)
        srcs = [SyntheticStereoSource(name=nm, scene=scene, trajectory=traj, rig_T_source=np.array(mats[nm]), seed=k,
                                      imu=(k == 0)) for k, nm in enumerate(names)]
        base_T_imu = np.array(mats[names[0]]) @ DRB_TO_RDF
        rig = CameraRig(srcs, rig_extrinsics={nm: Extrinsics.from_4x4_matrix(np.array(mats[nm])) for nm in names},
                        imu_source=names[0], imu_extrinsics=IMUExtrinsics(names[0], Extrinsics.from_4x4_matrix(base_T_imu)))
        rig.start()
        eng = HipSlamEngine(num_cameras=4, config=HipSlamConfig(batch_size=4, ba_window=4, ba_kf_interval=2, ba_iters=3,
                                                                enable_loop_closure=False, ba_inertial=inertial))
        eng.initialize(rig.calibration)
        calls = []
        inner = eng._handle.ba_inertial_factor
        eng._handle.ba_inertial_factor = lambda g, rec, v0, pair=0: (calls.append((g, pair)), inner(g, rec, v0, pair))
        for _ in range(n):
            eng.process_frames(rig.get_synchronized_frames())
        eng.flush()
        smap = eng.get_map()
        ine = eng._handle.ba_read_inertial(2) if inertial else None
        frames = eng._handle.ba_read(2)["frames"]
        eng.shutdown()
        pos_err = []
        for kf in smap.keyframe_poses:
            k = min(range(n), key=lambda i: abs(srcs[0].timestamp(i) - kf.timestamp))
            gt = np.linalg.inv(traj[0]) @ traj[k]
            pos_err.append(np.linalg.norm(kf.to_4x4_matrix()[:3, 3] - gt[:3, 3]))
        return calls, pos_err, ine, frames, traj, srcs[0]

    calls, err_on, ine, frames, traj, src = run(True)
    assert calls == [(g, 2) for g in (2, 4, 6, 8, 10, 12, 14)], calls
    assert np.isfinite(ine["vel"]).all() and np.isfinite(ine["bias"]).all()
    dt = 1.0 / src.fps
    for s, g in enumerate(frames):
        if g <= 0:
            continue
        v_true = (traj[int(g) + 1][:3, 3] - traj[int(g) - 1][:3, 3]) / (2 * dt)
        assert abs(np.linalg.norm(ine["vel"][s]) - np.linalg.norm(v_true)) < 0.05, (g, ine["vel"][s], v_true)
    calls_off, err_off, _, _, _, _ = run(False)
    assert calls_off == []
    assert len(err_on) == len(err_off) > 0
    assert max(err_on) < max(err_off) + 5e-3, (err_on, err_off)


def test_engine_ba_recovers_a_true_gyro_bias():
    """a synthetic IMU whose gyroscope reads a true bias of (0.02, -0.015, 0.01)
    rad/s.  The local BA window (accelerometer leg on: each record carries the gyro rotation rows,
    the bias Jacobians and both random walks) estimates a gyroscope bias per keyframe; after 60
    frames every window keyframe's estimate (IMU axes) is at least as close to the true bias as the
    host filter's (which fed the records' linearisation point and the oldest keyframe's prior), and
    the newest keyframe's is within 25 % of it."""
    from thor_slam_amd.camera import CameraRig, Extrinsics
    from thor_slam_amd.camera.types import IMUExtrinsics
    from thor_slam_amd.params import HipSlamConfig
    from thor_slam_amd.slam.hip_engine import HipSlamEngine
    from thor_slam_amd.synthetic import DRB_TO_RDF, SyntheticStereoSource

    bg_true = np.array([0.02, -0.015, 0.01])
    src = SyntheticStereoSource(seed=0, imu=True, n_frames=80, gyro_bias=bg_true)
    rig_T = src.rig_T_source
    rig = CameraRig([src], rig_extrinsics={src.name: Extrinsics.from_4x4_matrix(rig_T)}, imu_source=src.name,
                    imu_extrinsics=IMUExtrinsics(src.name, Extrinsics.from_4x4_matrix(rig_T @ DRB_TO_RDF)))
    rig.start()
    eng = HipSlamEngine(num_cameras=2, config=HipSlamConfig(batch_size=5, ba_window=6, ba_kf_interval=5, ba_iters=5,
                                                            enable_loop_closure=False))
    eng.initialize(rig.calibration)
    for _ in range(60):
        eng.process_frames(rig.get_synchronized_frames())
    eng.flush()
    ine = eng._handle.ba_read_inertial(0)
    frames = eng._handle.ba_read(0)["frames"]
    filt_bg = eng._imu.st.bg.copy()
    eng.shutdown()
    order = [s_ for s_ in np.argsort(frames) if frames[s_] >= 0]   # slots, oldest keyframe first
    est = ine["bias"][order][:, 3:6]
    err = np.abs(est - bg_true).max(axis=1)
    err_f = np.abs(filt_bg - bg_true).max()
    print(f"window gyro biases {est.round(4).tolist()} vs true {bg_true.tolist()} (filter: {filt_bg.round(4).tolist()})")
    assert len(order) == 6 and (err <= err_f + 1e-4).all(), (err, err_f)
    assert err[-1] < 0.25 * np.abs(bg_true).max(), (est[-1], bg_true)
