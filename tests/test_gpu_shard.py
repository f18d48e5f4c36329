"""Sharded rig: one camera stream per GPU, RCCL all-to-all of raw images + stream
blocks, per-pair A6/A7 + rig pose on each rank's frame range, all-gather of pose records.

Every rank must end each batch with exactly (bit for bit) the per-pair and rig poses of one
unsharded handle fed all cameras (which tests/test_gpu_rig.py checks against the oracle), and
the ring slots a rank imported must hold the other ranks' keypoints byte for byte.  The ranks
run in one process on one GPU (LocalShardedRig: the collectives become device copies; the
handles, kernels and buffers are the ones the multi-process path uses);
test_dist_shard_gloo_two_processes runs the real torch.distributed path with 2 processes.
"""

from __future__ import annotations

import json
import os
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

from helpers import C3_SOURCES, rig_scene
from thor_slam_amd.params import HipSlamConfig

pytestmark = pytest.mark.gpu
TWO = ("192.168.2.21", "192.168.2.25")
ROOT = Path(__file__).resolve().parents[1]


def unsharded(sc, cfg, batch, n_batches):
    import torch

    from thor_slam_amd._lib import Handle

    h = Handle(sc["rects"], cfg, max_batch=batch)
    h.set_rig(sc["E"])
    dev = torch.from_numpy(np.ascontiguousarray(sc["frames"])).cuda()
    out = []
    for b in range(n_batches):
        h.submit(dev[b * batch].data_ptr(), batch, torch.cuda.current_stream().cuda_stream)
        out.append({"pairs": h.read_poses(batch), "rig": h.read_rig_poses(batch)})
    kps = h.keypoints(n_batches * batch - 1, 0)
    h.close()
    return out, kps


def assert_identical(got, want):
    for part in ("pairs", "rig"):
        for k in ("T_rel", "T_abs", "cov", "stats"):
            np.testing.assert_array_equal(got[part][k], want[part][k], err_msg=f"{part}.{k}")


@pytest.mark.parametrize("world,exchange", [(2, "alltoall"), (4, "alltoall"), (4, "allgather")])
def test_sharded_two_pair_rig_identical(world, exchange):
    """4 cameras over 2 ranks (a pair per rank) or 4 ranks (one stream per rank), 3 batches."""
    import torch

    from thor_slam_amd.shard import LocalShardedRig

    batch, nb = 4, 3
    sc = rig_scene(TWO, batch * nb)
    cfg = HipSlamConfig()
    want, kps = unsharded(sc, cfg, batch, nb)
    rig = LocalShardedRig(sc["rects"], cfg, world=world, batch=batch, base_T_rect=sc["E"], exchange=exchange)
    dev = torch.from_numpy(np.ascontiguousarray(sc["frames"])).cuda()
    for b in range(nb):
        rig.step(dev[b * batch:(b + 1) * batch])
        for r in range(world):
            assert_identical(rig.read(r), want[b])
    assert (want[-1]["rig"]["stats"][:, 0] == 0).all()
    # the last rank solves the batch's last frame: camera 0's keypoints there came over the exchange
    got = rig.ranks[world - 1].h.keypoints(nb * batch - 1, 0)
    for k in ("x", "y", "level", "score", "counts"):
        np.testing.assert_array_equal(got[k], kps[k])
    rig.close()


def test_sharded_c3_one_stream_per_rank_identical():
    """C3 (BASELINE.json configs[2]): the four OAK sources of run_slam.py:45-50, 8 streams, one
    stream per rank on 8 ranks, 2 batches of 8 frames, identical to the unsharded rig."""
    import torch

    from thor_slam_amd.shard import LocalShardedRig

    batch, nb = 8, 2
    sc = rig_scene(C3_SOURCES, batch * nb)
    cfg = HipSlamConfig()
    want, _ = unsharded(sc, cfg, batch, nb)
    rig = LocalShardedRig(sc["rects"], cfg, world=8, batch=batch, base_T_rect=sc["E"])
    dev = torch.from_numpy(np.ascontiguousarray(sc["frames"])).cuda()
    for b in range(nb):
        rig.step(dev[b * batch:(b + 1) * batch])
        for r in (0, 3, 7):
            assert_identical(rig.read(r), want[b])
    assert (want[-1]["rig"]["stats"][:, 0] == 0).all()
    rig.close()


def test_dist_shard_gloo_two_processes(tmp_path):
    """The torch.distributed path (DistShardedRig) with 2 processes on this GPU, gloo (host-staged
    collectives), 2 pairs, one pair per rank, 2 batches: both ranks == the unsharded handle."""
    batch, nb = 4, 2
    sc = rig_scene(TWO, batch * nb)
    want, _ = unsharded(sc, HipSlamConfig(), batch, nb)
    env = dict(os.environ, PYTHONPATH=f"{ROOT}:{ROOT / 'thor-slam_amd'}:{ROOT / 'tests'}")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr=127.0.0.1",
           "--master-port=29517", str(ROOT / "tests" / "shard_worker.py"), str(tmp_path), str(batch), str(nb)]
    subprocess.run(cmd, check=True, env=env, timeout=240)
    for r in range(2):
        got = json.loads((tmp_path / f"rank{r}.json").read_text())
        for b in range(nb):
            for part in ("pairs", "rig"):
                for k in ("T_rel", "T_abs", "stats"):
                    np.testing.assert_array_equal(np.array(got[b][part][k]), want[b][part][k], err_msg=f"{r} {b} {part}.{k}")


def test_dist_shard_rccl_world_one(tmp_path):
    """DistShardedRig on the nccl (RCCL) backend, the bench's multi-GPU path, with one process:
    the all-to-all of images and stream blocks, the pose all-gather on its own communicator and
    the stream / event ordering between them must reproduce the unsharded handle bit for bit
    (more ranks need more GPUs than the test box has: RCCL refuses two ranks on one device)."""
    batch, nb = 4, 3
    sc = rig_scene(TWO, batch * nb)
    want, _ = unsharded(sc, HipSlamConfig(), batch, nb)
    env = dict(os.environ, PYTHONPATH=f"{ROOT}:{ROOT / 'thor-slam_amd'}:{ROOT / 'tests'}")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1", "--master-addr=127.0.0.1",
           "--master-port=29519", str(ROOT / "tests" / "shard_worker.py"), str(tmp_path), str(batch), str(nb), "nccl"]
    subprocess.run(cmd, check=True, env=env, timeout=240)
    got = json.loads((tmp_path / "rank0.json").read_text())
    for b in range(nb):
        for part in ("pairs", "rig"):
            for k in ("T_rel", "T_abs", "stats"):
                np.testing.assert_array_equal(np.array(got[b][part][k]), want[b][part][k], err_msg=f"{b} {part}.{k}")


def test_rccl_driven_shard_world_one_identical():
    """The library's own RCCL driver (tslam_comm_init + tslam_submit_sharded) on a
    1-rank communicator: the sharded stage runner over the whole range, the pose-record pack /
    ncclAllGather / unpack and the chain must reproduce the unsharded handle bit for bit (more
    ranks need more GPUs than the test box has: RCCL refuses two ranks on one device)."""
    import torch

    from thor_slam_amd._lib import Handle, comm_unique_id

    sc = rig_scene(names=TWO, n=12)
    cfg = HipSlamConfig()
    batch, nb = 4, 3
    want, _ = unsharded(sc, cfg, batch, nb)
    h = Handle(sc["rects"], cfg, max_batch=batch)
    h.set_rig(sc["E"])
    h.comm_init(comm_unique_id(), 0, 1)
    dev = torch.from_numpy(np.ascontiguousarray(sc["frames"])).cuda()
    s = torch.cuda.current_stream().cuda_stream
    for b in range(nb):
        h.submit_sharded(dev[b * batch].data_ptr(), stream=s)
        got = {"pairs": h.read_poses(batch), "rig": h.read_rig_poses(batch)}
        assert_identical(got, want[b])
    assert (want[-1]["rig"]["stats"][:, 0] == 0).all()
    h.close()


def _group_run(sc, cfg, world, batch, nb, transport):
    import torch

    from thor_slam_amd._lib import Handle, HandleGroup

    hs = [Handle(sc["rects"], cfg, max_batch=batch) for _ in range(world)]
    for h in hs:
        h.set_rig(sc["E"])
    grp = HandleGroup(hs, transport)
    S = sc["frames"].shape[1] // world
    parts = [torch.from_numpy(np.ascontiguousarray(sc["frames"][:, r * S:(r + 1) * S])).cuda() for r in range(world)]
    out = []
    for b in range(nb):
        grp.submit([p[b * batch].data_ptr() for p in parts])
        out.append([{"pairs": h.read_poses(batch), "rig": h.read_rig_poses(batch)} for h in hs])
    grp.close()
    for h in hs:
        h.close()
    return out


@pytest.mark.parametrize("world", [2, 4])
def test_library_driver_copy_transport_identical(world):
    """The library's own sharded driver (tslam_group_*: the code behind tslam_submit_sharded) with
    world ranks on this GPU and device copies for the collectives: raw-image staging per peer,
    stream-block packing, imports, double-buffered exchange buffers, pose records and the chain ==
    the unsharded handle, bit for bit, over 3 batches."""
    batch, nb = 4, 3
    sc = rig_scene(TWO, batch * nb)
    cfg = HipSlamConfig()
    want, _ = unsharded(sc, cfg, batch, nb)
    got = _group_run(sc, cfg, world, batch, nb, "copy")
    for b in range(nb):
        for r in range(world):
            assert_identical(got[b][r], want[b])


def test_library_driver_c3_eight_ranks_identical():
    """C3 through the library driver: 8 streams, one per rank, 8 ranks (copy transport)."""
    batch, nb = 8, 2
    sc = rig_scene(C3_SOURCES, batch * nb)
    cfg = HipSlamConfig()
    want, _ = unsharded(sc, cfg, batch, nb)
    got = _group_run(sc, cfg, 8, batch, nb, "copy")
    for b in range(nb):
        for r in (0, 5, 7):
            assert_identical(got[b][r], want[b])


def test_library_driver_rccl_clique_one_device():
    """tslam_group_create(RCCL): ncclCommInitAll clique (one device here), grouped sends /
    receives and the all-gather on the pose communicator == the unsharded handle."""
    batch, nb = 4, 3
    sc = rig_scene(TWO, batch * nb)
    cfg = HipSlamConfig()
    want, _ = unsharded(sc, cfg, batch, nb)
    got = _group_run(sc, cfg, 1, batch, nb, "rccl")
    for b in range(nb):
        assert_identical(got[b][0], want[b])


def test_sharded_batch_may_be_uneven():
    """tslam_begin_batch takes any batch length on a sharded handle (ranges of a 3-frame batch
    over 2 ranks: 1 and 2 frames; tests/test_gpu_shard_driver.py runs such batches)."""
    from thor_slam_amd._lib import Handle

    sc = rig_scene(TWO, 4)
    h = Handle(sc["rects"], HipSlamConfig(), max_batch=4)
    h.set_shard(0, 2, 0, 2)
    h.begin_batch(1 << 20, 3)   # accepted (nothing launched)
    h.end_batch()
    h.close()


def test_library_driver_short_batches_identical():
    """Batches of 4, 8 and 4 frames through a max_batch-8 group of 4 ranks (the per-batch frame
    ranges, per-peer slots and the all-gather shrink with the batch) == the unsharded handle fed
    the same batches."""
    import torch

    from thor_slam_amd._lib import Handle, HandleGroup

    sizes = [4, 8, 4]
    sc = rig_scene(TWO, sum(sizes))
    cfg = HipSlamConfig()
    h1 = Handle(sc["rects"], cfg, max_batch=8)
    h1.set_rig(sc["E"])
    hs = [Handle(sc["rects"], cfg, max_batch=8) for _ in range(4)]
    for h in hs:
        h.set_rig(sc["E"])
    grp = HandleGroup(hs, "copy")
    dev = torch.from_numpy(np.ascontiguousarray(sc["frames"])).cuda()
    parts = [dev[:, r:r + 1].contiguous() for r in range(4)]
    f0 = 0
    for n in sizes:
        h1.submit(dev[f0].data_ptr(), n, torch.cuda.current_stream().cuda_stream)
        want = {"pairs": h1.read_poses(n), "rig": h1.read_rig_poses(n)}
        grp.submit([p[f0].data_ptr() for p in parts], n)
        for h in hs:
            assert_identical({"pairs": h.read_poses(n), "rig": h.read_rig_poses(n)}, want)
        f0 += n
    grp.close()
    for h in hs + [h1]:
        h.close()
