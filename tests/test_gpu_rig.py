"""Rig pose: generalised PnP over every pair of a multi-source rig,
HIP ``k_rig_pose`` vs ``oracle/numpy_rig.py`` on the two-source bracket rig.

Bar: status and the winning candidate identical, inlier counts within 2 (the candidates start
from per-pair poses that agree with the oracle to ~1e-16, so a borderline inlier may flip), body
motions and chained world_T_base within 1e-9 relative Frobenius.
"""

from __future__ import annotations

import functools
import json
from pathlib import Path

import numpy as np
import pytest

from helpers import rel_frobenius
from oracle import numpy_slam as O
from oracle.numpy_rig import RigChain, rig_pose
from thor_slam_amd.calib import extract_cameras, stereo_pairs, stereo_rectify
from thor_slam_amd.camera import CameraRig, Extrinsics
from thor_slam_amd.params import HipSlamConfig
from thor_slam_amd.synthetic import RoomScene, SyntheticStereoSource, circle_trajectory

pytestmark = pytest.mark.gpu
NAMES = ["192.168.2.21", "192.168.2.25"]


@functools.lru_cache(maxsize=2)
def rig_scenario(n: int = 6):
    mats = json.loads((Path(__file__).parent / "golden" / "brackets_joints.json").read_text())
    scene = RoomScene(seed=0)
    traj = circle_trajectory(40)
    srcs = [SyntheticStereoSource(name=nm, scene=scene, trajectory=traj, rig_T_source=np.array(mats[nm]), seed=k)
            for k, nm in enumerate(NAMES)]
    rig = CameraRig(srcs, rig_extrinsics={nm: Extrinsics.from_4x4_matrix(np.array(mats[nm])) for nm in NAMES})
    cams = extract_cameras(rig.calibration, 4)
    pairs = stereo_pairs(cams)
    rects = [stereo_rectify(cams[l], cams[r]) for l, r in pairs]
    E = [cams[l].extrinsics.to_4x4_matrix() @ r.left_optical_T_rect() for (l, _), r in zip(pairs, rects)]
    by_name = {s.name: s for s in srcs}
    frames = np.stack([np.stack([by_name[cams[l].source_name].render_image(i, c) for l, _ in pairs for c in (0, 1)])
                       for i in range(n)])   # [n][4][H][W]
    cfg = HipSlamConfig()
    trks = [O.OracleTracker(cfg, dict(fx=r.fx, fy=r.fy, cx=r.cx, cy=r.cy, baseline=r.baseline, map_l=r.map_left,
                                      map_r=r.map_right)) for r in rects]
    chain = RigChain()
    want = []
    for i in range(n):
        outs = [trk.step(frames[i, 2 * q], frames[i, 2 * q + 1]) for q, trk in enumerate(trks)]
        if i == 0:
            want.append({"status": 2, "T_abs": np.eye(4)})
            continue
        items = [{"status": o["status"], "T": o["T"], "corr": o.get("corr"),
                  "intr": (r.fx, r.fy, r.cx, r.cy)} for o, r in zip(outs, rects)]
        res = rig_pose(items, E, cfg)
        res["T_abs"] = chain.step(res)
        want.append(res)
    return {"frames": frames, "rects": rects, "E": E, "cfg": cfg, "want": want, "traj": traj}


@pytest.mark.parametrize("batch", [6, 2])
def test_rig_pose_matches_oracle(batch):
    import torch

    from thor_slam_amd._lib import Handle

    sc = rig_scenario()
    h = Handle(sc["rects"], sc["cfg"], max_batch=batch)
    h.set_rig(sc["E"])
    dev = torch.from_numpy(np.ascontiguousarray(sc["frames"])).cuda()
    n = dev.shape[0]
    got = []
    for b0 in range(0, n, batch):
        nb = min(batch, n - b0)
        h.submit(dev[b0:].data_ptr(), nb, torch.cuda.current_stream().cuda_stream)
        r = h.read_rig_poses(nb)
        got += [{k: r[k][f] for k in r} for f in range(nb)]
    h.close()
    for i, (g, w) in enumerate(zip(got, sc["want"])):
        assert g["stats"][0] == w["status"], i
        if i == 0:
            continue
        assert g["stats"][4] == w["best"] and abs(int(g["stats"][2]) - w["n_inliers"]) <= 2, (i, g["stats"], w)
        assert rel_frobenius(g["T_rel"], w["T"]) < 1e-9, i
        assert rel_frobenius(g["T_abs"], w["T_abs"]) < 1e-9, i
        assert rel_frobenius(g["cov"], w["cov"]) < 1e-6, i
    # and the joint solve tracks the rendered body motion
    gt = np.linalg.inv(sc["traj"][0]) @ sc["traj"][n - 1]
    assert np.linalg.norm(got[-1]["T_abs"][:3, 3] - gt[:3, 3]) < 0.1 * np.linalg.norm(gt[:3, 3]) + 2e-3


def test_rig_pose_survives_a_blind_pair():
    """One pair sees a blank wall (no correspondences): the rig still tracks from the other."""
    import torch

    from thor_slam_amd._lib import Handle

    sc = rig_scenario()
    frames = sc["frames"].copy()
    frames[:, 2:] = 128   # pair 1 blind
    h = Handle(sc["rects"], sc["cfg"], max_batch=6)
    h.set_rig(sc["E"])
    dev = torch.from_numpy(np.ascontiguousarray(frames)).cuda()
    h.submit(dev.data_ptr(), 6, torch.cuda.current_stream().cuda_stream)
    r = h.read_rig_poses(6)
    per = h.read_poses(6)
    h.close()
    assert (per["stats"][1:, 1, 0] != 0).all()          # the blind pair is lost
    assert (r["stats"][1:, 0] == 0).all()               # the rig is not
    gt = np.linalg.inv(sc["traj"][0]) @ sc["traj"][5]
    assert np.linalg.norm(r["T_abs"][5][:3, 3] - gt[:3, 3]) < 0.1 * np.linalg.norm(gt[:3, 3]) + 2e-3


def test_rig_fusion_across_ranks_matches_numpy():
    """Multi-GPU layout rehearsed on one GPU: one handle per pair ("rank"), their packed blocks
    concatenated as the all-gather would, fused on the device (tslam_rig_fuse) vs numpy."""
    import torch

    from oracle.numpy_rig import RigChain, fuse_information
    from thor_slam_amd._lib import Handle

    sc = rig_scenario()
    n = 6
    stream = torch.cuda.current_stream().cuda_stream
    handles, blocks, per = [], [], []
    for q in range(2):
        h = Handle([sc["rects"][q]], sc["cfg"], max_batch=n)
        dev = torch.from_numpy(np.ascontiguousarray(sc["frames"][:, 2 * q:2 * q + 2])).cuda()
        h.submit(dev.data_ptr(), n, stream)
        per.append(h.read_poses(n))
        blk = torch.empty(64 << 20, dtype=torch.uint8, device="cuda")
        nb = h.pack_features(blk.data_ptr(), stream)
        blocks.append(blk[:nb])
        handles.append(h)
    gathered = torch.cat(blocks).contiguous()
    h0 = handles[0]
    h0.set_rig_ranks(sc["E"])
    h0.rig_fuse(gathered.data_ptr(), 2, 0, n, stream)
    got = h0.read_rig_poses(n)
    for h in handles:
        h.close()
    chain = RigChain()
    for f in range(n):
        items = [(int(per[q]["stats"][f, 0, 0]), per[q]["T_rel"][f, 0], per[q]["cov"][f, 0]) for q in range(2)]
        w = fuse_information(items, sc["E"])
        w_abs = chain.step(w)
        assert got["stats"][f, 0] == w["status"], f
        if w["status"] == 0:
            assert got["stats"][f, 1] == w["used"] == 2
            assert rel_frobenius(got["T_rel"][f], w["T"]) < 1e-9
            assert rel_frobenius(got["cov"][f], w["cov"]) < 1e-6
        assert rel_frobenius(got["T_abs"][f], w_abs) < 1e-9
    gt = np.linalg.inv(sc["traj"][0]) @ sc["traj"][n - 1]
    assert np.linalg.norm(got["T_abs"][n - 1][:3, 3] - gt[:3, 3]) < 0.1 * np.linalg.norm(gt[:3, 3]) + 2e-3
