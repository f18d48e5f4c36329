"""RGB-D input (BASELINE.json configs[4]): HIP path vs the oracle's ``step_rgbd`` on identical frames.

Bar: keypoints / descriptors / temporal matches bit-exact (same integer path as stereo), the
depth-derived disparities bit-exact (same IEEE ops), poses within 1e-9 relative Frobenius.
"""

from __future__ import annotations

import functools

import numpy as np
import pytest

from helpers import DISTORTION, rel_frobenius
from oracle import numpy_slam as O
from thor_slam_amd.calib import extract_cameras, rgbd_pairs, rgbd_undistort
from thor_slam_amd.camera.rig import CameraRig
from thor_slam_amd.params import HipSlamConfig
from thor_slam_amd.synthetic import SyntheticRGBDSource

pytestmark = pytest.mark.gpu


@functools.lru_cache(maxsize=4)
def rgbd_scenario(n: int = 4, width: int = 640, height: int = 400, distorted: bool = False, features: int = 2000):
    src = SyntheticRGBDSource(width=width, height=height, distortion=DISTORTION if distorted else None)
    cams = extract_cameras(CameraRig([src]).calibration, 2)
    (ci, _), = rgbd_pairs(cams)
    rect = rgbd_undistort(cams[ci])
    cfg = HipSlamConfig(rgbd=True, n_features=features)
    trk = O.OracleTracker(cfg, dict(fx=rect.fx, fy=rect.fy, cx=rect.cx, cy=rect.cy, baseline=rect.baseline,
                                    map_l=rect.map_left, map_r=rect.map_right))
    frames = [src.render_rgbd(i) for i in range(n)]
    oracle = [trk.step_rgbd(b, d) for b, d in frames]
    records = src.render_rgbd_sequence(n)[:, None, :]   # [n][1 camera][5*H*W]
    return {"src": src, "rect": rect, "cfg": cfg, "oracle": oracle, "records": records}


def _hip(sc, batch):
    import torch

    from thor_slam_amd._lib import Handle

    h = Handle([sc["rect"]], sc["cfg"], max_batch=batch)
    dev = torch.from_numpy(np.ascontiguousarray(sc["records"])).cuda()
    n = dev.shape[0]
    K = sc["cfg"].n_features
    out = []
    for b0 in range(0, n, batch):
        nb = min(batch, n - b0)
        h.submit(dev[b0:].data_ptr(), nb, torch.cuda.current_stream().cuda_stream)
        res = h.read_poses(nb)
        for f in range(nb):
            g = b0 + f
            slot = h.ring_slot(g)
            out.append({"kp": h.keypoints(g, 0), "disp": h.frame_block("disp", slot, np.float64)[:K],
                        "stereo": h.frame_block("stereo", slot, np.int32)[:K],
                        "temporal": h.frame_block("temporal", slot, np.int32)[:K],
                        "T_abs": res["T_abs"][f, 0], "stats": res["stats"][f, 0]})
    h.close()
    return out


def _check(sc, got):
    for i, (rec, o) in enumerate(zip(got, sc["oracle"])):
        left = o["cur"]["left"]
        kp = left["kp"]
        np.testing.assert_array_equal(rec["kp"]["counts"], left["counts"], err_msg=f"frame {i}")
        for k in ("x", "y", "score", "angle", "level"):
            np.testing.assert_array_equal(rec["kp"][k][left["valid"]], kp[k][left["valid"]], err_msg=f"frame {i} {k}")
        np.testing.assert_array_equal(rec["kp"]["desc"][left["valid"]], left["desc"][left["valid"]])
        np.testing.assert_array_equal(rec["disp"], o["cur"]["disp"], err_msg=f"frame {i} disp")
        np.testing.assert_array_equal(rec["stereo"], o["cur"]["stereo"])
        np.testing.assert_array_equal(rec["temporal"], o["cur"]["temporal"])
        if i:
            assert rec["stats"][0] == o["status"] and rec["stats"][2] == o["n_inliers"]
            assert rel_frobenius(rec["T_abs"], o["world_T_cam"]) < 1e-9


@pytest.mark.parametrize("batch", [4, 1])
def test_rgbd_bit_exact(batch):
    sc = rgbd_scenario()
    _check(sc, _hip(sc, batch))
    assert all(o["status"] == 0 for o in sc["oracle"][1:])


def test_rgbd_distorted_lens_bit_exact():
    """Undistortion map on the colour image and on the depth lookup."""
    sc = rgbd_scenario(n=3, distorted=True)
    assert not sc["rect"].is_identity
    _check(sc, _hip(sc, 3))


def test_rgbd_c5_size():
    """Config C5 geometry: 1280x720 colour + depth, K=4000."""
    sc = rgbd_scenario(n=2, width=1280, height=720, features=4000)
    _check(sc, _hip(sc, 2))


def test_engine_rgbd_matches_oracle():
    from thor_slam_amd.camera import Extrinsics
    from thor_slam_amd.slam.hip_engine import HipSlamEngine

    sc = rgbd_scenario()
    src = SyntheticRGBDSource(width=640, height=400)
    rig = CameraRig([src], rig_extrinsics={src.name: Extrinsics.from_4x4_matrix(src.rig_T_source)})
    rig.start()
    # sync: each call returns its own frame's pose (the asynchronous default may lag)
    eng = HipSlamEngine(num_cameras=2, config=HipSlamConfig(rgbd=True, sync=True))
    eng.initialize(rig.calibration)
    bt = src.rig_T_source @ src.get_extrinsics()[0].to_4x4_matrix() @ sc["rect"].left_optical_T_rect()
    for i in range(4):
        pose = eng.process_frames(rig.get_synchronized_frames())
        want = bt @ sc["oracle"][i]["world_T_cam"] @ np.linalg.inv(bt)
        assert rel_frobenius(pose.to_4x4_matrix(), want) < 1e-9
    gt = np.linalg.inv(src.ground_truth_body(0)) @ src.ground_truth_body(3)
    assert np.linalg.norm(pose.position - gt[:3, 3]) < 0.1 * np.linalg.norm(gt[:3, 3]) + 2e-3
    eng.shutdown()
