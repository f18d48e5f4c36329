"""Map persistence + relocalisation: the A8 window's landmarks carry the
descriptors of their keyframe keypoints; a map built from them relocalises a frame of a fresh
handle.  HIP ``k_reloc`` vs ``oracle/numpy_map.py``: matches, RANSAC winner and inlier counts
identical, cam_T_world within 1e-9 relative Frobenius."""

from __future__ import annotations

import numpy as np
import pytest

from helpers import rel_frobenius
from oracle.numpy_map import relocalize
from test_gpu_ba import _scenario_and_oracle

pytestmark = pytest.mark.gpu


def _oracle_map(sc, want):
    """Landmarks of the oracle's final window: world xyz (rect frame 0) + keyframe descriptors."""
    K = sc["cfg"].n_features
    w = want[-1]
    ids = np.unique(w["lm"][w["frames"] >= 0])
    ids = ids[ids >= 0]
    desc = np.stack([sc["oracle"][int(w["frames"][i // K])]["cur"]["left"]["desc"][i % K] for i in ids])
    return ids, w["X"][ids], desc.astype(np.uint32)


def test_window_map_descriptors_and_relocalisation():
    import torch

    from thor_slam_amd._lib import Handle
    from thor_slam_amd.params import HipSlamConfig

    sc, want = _scenario_and_oracle(12)
    ids, xyz, desc = _oracle_map(sc, want)
    # 1. the device window exports the same map (descriptors bit-exact, positions to 1e-9)
    h = Handle([sc["rect"]], sc["cfg"], max_batch=12)
    dev = torch.from_numpy(np.ascontiguousarray(sc["frames"])).cuda()
    h.submit(dev.data_ptr(), 12, torch.cuda.current_stream().cuda_stream)
    win, mp = h.ba_read(0), h.ba_read_map(0)
    h.close()
    np.testing.assert_array_equal(mp["desc"][ids], desc)
    assert np.abs(win["X"][ids] - xyz).max() < 1e-9 * np.abs(xyz).max()
    gids = mp["gid"][ids]
    assert np.unique(gids).size == gids.size and (gids >= 0).all()
    # 2. relocalise frames of a fresh handle (no BA) against that map
    cfg = HipSlamConfig()
    rect = sc["rect"]
    intr = (rect.fx, rect.fy, rect.cx, rect.cy)
    h = Handle([rect], cfg, max_batch=4)
    h.map_upload(xyz, desc)
    h.submit(dev[8:].data_ptr(), 4, torch.cuda.current_stream().cuda_stream)   # frames 8..11 as 0..3
    for f in range(4):
        got = h.relocalize(f)
        o = relocalize(sc["oracle"][8 + f]["cur"]["left"], xyz, desc, intr, cfg, f)
        assert got["stats"][0] == o["status"] == 0, (f, got["stats"])
        assert got["stats"][1] == o["n_corr"] and got["stats"][2] == o["n_inliers"] and got["stats"][4] == o["best_hyp"]
        assert rel_frobenius(got["T"], o["T"]) < 1e-9
        # the map frame is rect-left of frame 0: cam_T_world ~ inv(front-end world_T_cam)
        fe = np.linalg.inv(sc["oracle"][8 + f]["world_T_cam"])
        assert np.linalg.norm(got["T"][:3, 3] - fe[:3, 3]) < 0.02
    h.close()


def test_relocalise_fails_cleanly_on_an_unrelated_map():
    import torch

    from thor_slam_amd._lib import Handle
    from thor_slam_amd.params import HipSlamConfig

    sc, _ = _scenario_and_oracle(12)
    rng = np.random.default_rng(0)
    h = Handle([sc["rect"]], HipSlamConfig(), max_batch=1)
    h.map_upload(rng.normal(size=(500, 3)), rng.integers(0, 2**32, size=(500, 8), dtype=np.uint32))
    dev = torch.from_numpy(np.ascontiguousarray(sc["frames"])).cuda()
    h.submit(dev.data_ptr(), 1, torch.cuda.current_stream().cuda_stream)
    got = h.relocalize(0)
    h.close()
    assert got["stats"][0] != 0 and np.array_equal(got["T"], np.eye(4))


def test_engine_save_load_relocalize(tmp_path):
    """Session 1 (local BA on) maps the room and saves it; session 2 loads the map, sees a later
    frame, relocalises, and from then on publishes poses in session 1's world frame."""
    from thor_slam_amd.camera import CameraRig, Extrinsics
    from thor_slam_amd.params import HipSlamConfig
    from thor_slam_amd.slam import TrackingState
    from thor_slam_amd.slam.hip_engine import HipSlamEngine

    from helpers import make_source
    from test_gpu_ba import BA_ITEMS

    def engine(cfg):
        src = make_source(0)
        rig = CameraRig([src], rig_extrinsics={src.name: Extrinsics.from_4x4_matrix(src.rig_T_source)})
        rig.start()
        eng = HipSlamEngine(num_cameras=2, config=cfg)
        eng.initialize(rig.calibration)
        return eng, rig

    eng, rig = engine(HipSlamConfig(**dict(BA_ITEMS)))
    assert eng.save_map(str(tmp_path / "empty.npz")) is False
    poses1 = [eng.process_frames(rig.get_synchronized_frames()) for _ in range(12)]
    path = str(tmp_path / "room.npz")
    assert eng.save_map(path)
    smap = eng.get_map()
    eng.shutdown()
    with np.load(path, allow_pickle=False) as z:
        assert z["points"].shape[0] == len(smap.points) or z["points"].shape[0] >= len(smap.points)
        assert z["desc"].dtype == np.uint32 and z["desc"].shape[1] == 8

    eng2, rig2 = engine(HipSlamConfig())
    assert eng2.relocalize() is False                # no map yet
    assert eng2.load_map(path)
    for _ in range(8):                               # session 2 starts at frame 8 of the same path
        rig2.get_synchronized_frames()
    p = eng2.process_frames(rig2.get_synchronized_frames())
    assert eng2.relocalize()
    assert eng2.get_tracking_state() == TrackingState.TRACKING
    p = eng2._latest_pose
    assert np.linalg.norm(p.position - poses1[8].position) < 0.02
    for k in range(9, 12):
        p = eng2.process_frames(rig2.get_synchronized_frames())
        assert np.linalg.norm(p.position - poses1[k].position) < 0.02, k
    assert eng2.load_map(str(tmp_path / "missing.npz")) is False
    eng2.shutdown()


def test_rig_relocalisation_from_a_map_seen_by_pair_1():
    """tslam_relocalize_rig on the two-source bracket rig: the map holds only pair 1's stereo
    landmarks of frame 0 (base frame), so pair 0 cannot pose itself — the rig still relocalises from
    pair 1's view through the rig pose.  Against oracle/numpy_map.relocalize_rig: every pair's
    status, matches, RANSAC winner and inliers and the rig's winner / inliers identical, body_T_world
    within 1e-9; and it equals the ground-truth body motion to 2 cm."""
    import torch

    from helpers import rig_scene
    from oracle import numpy_slam as O
    from oracle.numpy_map import relocalize_rig
    from thor_slam_amd._lib import Handle
    from thor_slam_amd.params import HipSlamConfig

    names = ("192.168.2.21", "192.168.2.25")
    n = 3
    sc = rig_scene(names, n)
    cfg = HipSlamConfig()
    rects, E = sc["rects"], sc["E"]
    trk = [O.OracleTracker(cfg, dict(fx=r.fx, fy=r.fy, cx=r.cx, cy=r.cy, baseline=r.baseline, map_l=r.map_left,
                                     map_r=r.map_right)) for r in rects]
    ora = [[trk[p].step(sc["frames"][f, 2 * p], sc["frames"][f, 2 * p + 1]) for p in range(len(rects))] for f in range(n)]
    # the map: pair 1's left keypoints of frame 0 with a disparity, in the base frame of frame 0
    r1, cur = rects[1], ora[0][1]["cur"]
    left, disp = cur["left"], cur["disp"]
    ok = left["valid"] & np.isfinite(disp) & (disp > 0)
    u, v = O.level0_coords(left["kp"]["x"][ok], left["kp"]["y"][ok], left["kp"]["level"][ok])
    z = r1.fx * r1.baseline / disp[ok]
    cam = np.stack([(u - r1.cx) * z / r1.fx, (v - r1.cy) * z / r1.fy, z, np.ones_like(z)])
    xyz = (np.asarray(E[1]) @ cam)[:3].T.copy()
    desc = left["desc"][ok].astype(np.uint32)
    assert xyz.shape[0] > 200
    h = Handle(rects, cfg, max_batch=n)
    h.set_rig(E)
    dev = torch.from_numpy(np.ascontiguousarray(sc["frames"])).cuda()
    h.submit(dev.data_ptr(), n, torch.cuda.current_stream().cuda_stream)
    h.map_upload(xyz, desc)
    g = n - 1
    got = h.relocalize_rig(g)
    h.close()
    intrs = [(r.fx, r.fy, r.cx, r.cy) for r in rects]
    want = relocalize_rig([ora[g][p]["cur"]["left"] for p in range(len(rects))], xyz, desc, intrs, E, cfg, g)
    for p, wp in enumerate(want["pairs"]):
        st = got["pair_stats"][p]
        assert st[0] == wp["status"] and st[1] == wp["n_corr"], (p, st, wp["status"], wp["n_corr"])
        if wp["status"] == 0:
            assert st[2] == wp["n_inliers"] and st[4] == wp["best_hyp"]
    assert got["pair_stats"][1][0] == 0 and got["pair_stats"][1][1] > 100   # pair 1 sees the map
    assert got["pair_stats"][0][1] < got["pair_stats"][1][1] // 4             # pair 0 hardly does
    st = got["stats"]
    assert st[0] == want["status"] == 0
    assert st[2] == want["n_inliers"] and st[4] == want["best"]
    assert rel_frobenius(got["T"], want["T"]) < 1e-9
    traj = sc["traj"]
    gt = np.linalg.inv(np.linalg.inv(traj[0]) @ traj[g])   # body_T_world, world = body at frame 0
    assert np.linalg.norm(got["T"][:3, 3] - gt[:3, 3]) < 0.02
