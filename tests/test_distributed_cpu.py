"""N>1 logic on CPU: the feature/pose block layout, the gloo all-gather of world_size 2, and the
rig-motion fusion (the GPU run uses the same code with the nccl=RCCL backend)."""

import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp
from scipy.spatial.transform import Rotation

from thor_slam_amd.dist import BlockLayout, FeatureExchange, body_motion, fuse_rig_motion, pack_block, unpack_rank_block

LAYOUT = BlockLayout(n_frames=3, n_cams=2, K=64, L=2)


def _block(rank: int) -> tuple[np.ndarray, dict]:
    rng = np.random.default_rng(100 + rank)
    lay = LAYOUT
    x = rng.integers(0, 640, size=(lay.n_frames, lay.n_cams, lay.K))
    y = rng.integers(0, 400, size=x.shape)
    lvl = rng.integers(0, lay.L, size=x.shape)
    kps = np.stack([x | (y << 16), lvl | (rng.integers(0, 30, size=x.shape) << 8)], -1).astype(np.uint32)
    desc = rng.integers(0, 2**32, size=(lay.n_frames, lay.n_cams, lay.K, 8), dtype=np.uint64).astype(np.uint32)
    counts = rng.integers(0, lay.K, size=(lay.n_frames, lay.n_cams, lay.L)).astype(np.int32)
    t_rel = np.tile(np.eye(4), (lay.n_frames, lay.n_pairs, 1, 1))
    t_rel[..., 0, 3] = rank + 0.5
    cov = rng.normal(size=(lay.n_frames, lay.n_pairs, 6, 6))
    stats = rng.integers(0, 100, size=(lay.n_frames, lay.n_pairs, 8)).astype(np.int32)
    return pack_block(lay, kps, desc, counts, t_rel, cov, stats), dict(x=x, y=y, desc=desc, counts=counts, t_rel=t_rel, cov=cov, stats=stats)


def test_block_roundtrip():
    buf, ref = _block(0)
    assert buf.size == LAYOUT.rank_bytes
    got = unpack_rank_block(LAYOUT, buf)
    np.testing.assert_array_equal(got["x"], ref["x"])
    np.testing.assert_array_equal(got["y"], ref["y"])
    np.testing.assert_array_equal(got["desc"], ref["desc"])
    np.testing.assert_array_equal(got["counts"], ref["counts"])
    np.testing.assert_array_equal(got["T_rel"], ref["t_rel"])
    np.testing.assert_array_equal(got["cov"], ref["cov"])
    np.testing.assert_array_equal(got["stats"], ref["stats"])


def _worker(rank: int, world: int, port: int, out_dir: str):
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ex = FeatureExchange(LAYOUT, "cpu", world)
    buf, _ = _block(rank)
    ex.send.copy_(torch.from_numpy(buf))
    ex.all_gather()
    ranks = ex.ranks()
    for r in range(world):
        _, ref = _block(r)
        np.testing.assert_array_equal(ranks[r]["desc"], ref["desc"])
        np.testing.assert_array_equal(ranks[r]["T_rel"], ref["t_rel"])
    open(os.path.join(out_dir, f"ok{rank}"), "w").write("ok")
    dist.destroy_process_group()


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_gloo_allgather_world2(tmp_path):
    mp.spawn(_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    assert (tmp_path / "ok0").exists() and (tmp_path / "ok1").exists()


def _rig():
    import json
    from pathlib import Path

    mats = json.loads((Path(__file__).parent / "golden" / "brackets_joints.json").read_text())
    return [np.array(m) for _, m in sorted(mats.items())]


def test_fuse_rig_motion_recovers_body_motion():
    rng = np.random.default_rng(3)
    motion = np.eye(4)
    motion[:3, :3] = Rotation.from_rotvec([0.01, -0.02, 0.03]).as_matrix()
    motion[:3, 3] = [0.02, -0.01, 0.005]
    cams = _rig()
    rels, covs = [], []
    for bt in cams:
        # cam_{t-1} -> cam_t point map consistent with the body motion
        cam_motion = np.linalg.inv(bt) @ motion @ bt
        rel = np.linalg.inv(cam_motion)
        np.testing.assert_allclose(body_motion(bt, rel), motion, atol=1e-12)
        noise = np.eye(4)
        noise[:3, :3] = Rotation.from_rotvec(rng.normal(0, 1e-4, 3)).as_matrix()
        noise[:3, 3] = rng.normal(0, 1e-4, 3)
        rels.append(rel @ noise)
        covs.append(np.eye(6) * 1e-8)
    fused = fuse_rig_motion(cams, rels, covs, [True] * len(cams))
    assert np.linalg.norm(fused[:3, 3] - motion[:3, 3]) < 5e-4
    assert np.linalg.norm(fused[:3, :3] - motion[:3, :3]) < 5e-4
    assert fuse_rig_motion(cams, rels, covs, [False] * len(cams)) is None
    # an unreliable source (huge covariance) barely moves the estimate
    bad = [r.copy() for r in rels]
    bad[0][:3, 3] += 0.5
    covs2 = [c.copy() for c in covs]
    covs2[0] = np.eye(6) * 1e6
    fused2 = fuse_rig_motion(cams, bad, covs2, [True] * len(cams))
    assert np.linalg.norm(fused2[:3, 3] - motion[:3, 3]) < 5e-3
