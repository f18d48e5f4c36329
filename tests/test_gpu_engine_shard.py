"""The sharded rig behind the ``SlamEngine`` boundary (cuVSLAM's multicam mode,
launch/thor_visual_slam.launch.py:49,81): ``HipSlamEngine`` with ``HipSlamConfig(devices=[...])``
owns one handle per device and drives them from one process as one sharded rig
(``tslam_group_*``).  The caller's loop is the reference's (scripts/run_slam.py:299-321:
``initialize(rig.calibration)`` then ``process_frames`` per synchronised set), unchanged.

Bar: every published ``SlamPose`` (position, quaternion, covariance, state, timestamp) is
bit-identical to the one-device engine's on the C3 rig (4 OAK sources, 8 streams) — through the
RCCL clique on one device, and with 4 or 8 ranks on this GPU over the copy transport — also with
local BA and loop closure on (the driver's state gather: rank 0 solves the window), for the short
last batch of a stream that does not fill batch_size x devices, and through relocalisation.
"""

from __future__ import annotations

import functools
import json
from pathlib import Path

import numpy as np
import pytest

from helpers import C3_SOURCES
from thor_slam_amd.camera import CameraRig, Extrinsics
from thor_slam_amd.params import HipSlamConfig
from thor_slam_amd.synthetic import RoomScene, SyntheticStereoSource, circle_trajectory

pytestmark = pytest.mark.gpu


@functools.lru_cache(maxsize=1)
def c3_frame_sets(n: int = 18):
    mats = json.loads((Path(__file__).parent / "golden" / "brackets_joints.json").read_text())
    scene = RoomScene(seed=0)
    traj = circle_trajectory(40)
    srcs = [SyntheticStereoSource(name=nm, scene=scene, trajectory=traj, rig_T_source=np.array(mats[nm]), seed=k)
            for k, nm in enumerate(C3_SOURCES)]
    rig = CameraRig(srcs, rig_extrinsics={nm: Extrinsics.from_4x4_matrix(np.array(mats[nm])) for nm in C3_SOURCES})
    rig.start()
    sets = [rig.get_synchronized_frames() for _ in range(n)]
    return rig.calibration, sets


def run_engine(cfg: HipSlamConfig, n: int = 16, extra: dict | None = None, map_path=None) -> list:
    """The latest pose after every published batch (process_frames' own return value depends on
    when the asynchronous one-device engine polls, so the per-batch publications are compared).
    ``extra`` (a dict) receives the map, the loop-closure graph and relocalize's outcome."""
    from thor_slam_amd.slam.hip_engine import HipSlamEngine

    cal, sets = c3_frame_sets()
    sets = sets[:n]
    eng = HipSlamEngine(num_cameras=8, config=cfg)
    eng.initialize(cal)
    published = []
    orig = eng._publish

    def record(res, stamps, g0):
        orig(res, stamps, g0)
        published.append(eng._latest_pose)

    eng._publish = record
    for fs in sets:
        eng.process_frames(fs)
    eng.flush()
    if extra is not None:
        smap = eng.get_map()
        extra["keyframes"] = [pose_tuple(p) for p in smap.keyframe_poses]
        extra["points"] = [(p.position.tobytes(), p.observations) for p in smap.points]
        extra["pose_graph"] = eng.pose_graph
        if map_path is not None:
            extra["relocalized"] = eng.load_map(str(map_path)) and eng.relocalize()
            extra["after_reloc"] = pose_tuple(eng._latest_pose)
        elif cfg.ba_window > 0:
            extra["saved"] = eng.save_map(str(extra["save_to"]))
    eng.shutdown()
    return published


def pose_tuple(p):
    if p is None:
        return None
    return (p.position.tobytes(), p.rotation.tobytes(), np.asarray(p.covariance).tobytes(), p.timestamp,
            p.tracking_state, p.confidence)


@pytest.mark.parametrize("devices,transport", [((0,), "rccl"), ((0,) * 8, "copy"), ((0,) * 4, "copy")])
def test_sharded_engine_poses_identical(devices, transport):
    base = HipSlamConfig(batch_size=8, enable_loop_closure=False)
    want = run_engine(base)
    got = run_engine(HipSlamConfig(batch_size=8, enable_loop_closure=False, devices=devices, shard_transport=transport))
    assert len(got) == len(want)
    assert [pose_tuple(p) for p in got] == [pose_tuple(p) for p in want]
    assert want[-1] is not None and want[-1].tracking_state.name == "TRACKING"


def test_sharded_engine_tracks_the_tail_of_a_stream():
    """18 frames over 8 ranks with batch_size 8: the third batch is the 2 trailing frames
    (submitted by flush as a short batch: six ranks have empty frame ranges); all three published
    batches equal the one-device engine's."""
    cfg = HipSlamConfig(batch_size=8, enable_loop_closure=False, devices=(0,) * 8, shard_transport="copy")
    got = run_engine(cfg, 18)
    want = run_engine(HipSlamConfig(batch_size=8, enable_loop_closure=False), 18)
    assert len(got) == len(want) == 3
    assert [pose_tuple(p) for p in got] == [pose_tuple(p) for p in want]


def test_sharded_engine_local_ba_and_loop_closure_identical(tmp_path):
    """devices=(0,)*4 over the copy transport on the C3 rig with a 10-keyframe local BA window and
    loop closure on, 18 frames in batches of 8 (the last 2 frames a short batch): every published
    pose, the map (BA keyframes and landmarks), the keyframe pose graph and the saved map equal the
    one-device engine's; then both relocalise the last frame in the one-device engine's map with the
    same outcome."""
    base = dict(batch_size=8, ba_window=10, enable_loop_closure=True)
    one, four = {"save_to": tmp_path / "one.npz"}, {"save_to": tmp_path / "four.npz"}
    want = run_engine(HipSlamConfig(**base), 18, one)
    got = run_engine(HipSlamConfig(**base, devices=(0,) * 4, shard_transport="copy"), 18, four)
    assert len(got) == len(want) == 3
    assert [pose_tuple(p) for p in got] == [pose_tuple(p) for p in want]
    assert want[-1] is not None and want[-1].tracking_state.name == "TRACKING"
    assert one["keyframes"] == four["keyframes"] and len(one["keyframes"]) >= 3
    assert one["points"] == four["points"] and len(one["points"]) > 100
    pg1, pg4 = one["pose_graph"], four["pose_graph"]
    assert pg1["frames"] == pg4["frames"] and len(pg1["frames"]) >= 3
    np.testing.assert_array_equal(pg1["T"], pg4["T"])
    assert one["saved"] and four["saved"]
    with np.load(one["save_to"]) as a, np.load(four["save_to"]) as b:
        for k in a.files:
            np.testing.assert_array_equal(a[k], b[k], err_msg=k)
    r1, r4 = {}, {}
    run_engine(HipSlamConfig(**base), 18, r1, map_path=one["save_to"])
    run_engine(HipSlamConfig(**base, devices=(0,) * 4, shard_transport="copy"), 18, r4, map_path=one["save_to"])
    assert r1["relocalized"] and r4["relocalized"]
    assert r1["after_reloc"] == r4["after_reloc"]
