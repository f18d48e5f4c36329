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
