"""The library's sharded-rig driver (tslam_shard.cpp) beyond full, evenly split batches:

* batches of any length 1 .. max_batch (uneven and empty frame ranges, raw images sent straight
  from the input, the padded pose all-gather);
* the state gather (TSLAM_SHARD_GATHER): rank 0's ring then holds every pair's temporal matches,
  disparities, left keypoints and descriptors as one handle's does, and rank 0 solves the local
  BA window — bit-identical to one handle fed all cameras;
* pinned result slots (TSLAM_SHARD_RESULTS: tslam_poll_batch on a sharded handle) and the
  per-segment HIP-event timing (TSLAM_SHARD_PROFILE);
* the pair split (TSLAM_SHARD_PAIRS): each rank solves its camera's pair over half the batch with
  the partner's images only, and the rig ranges gather pair blocks — identical results.

Ranks share this GPU through the COPY transport (the same packing, ordering and buffers as RCCL);
the RCCL transport runs at world 1 (one device on the test box)."""

from __future__ import annotations

import numpy as np
import pytest

from helpers import C3_SOURCES, rig_scene
from thor_slam_amd.params import HipSlamConfig

pytestmark = pytest.mark.gpu
TWO = ("192.168.2.21", "192.168.2.25")


def _poses(h, n):
    return {"pairs": h.read_poses(n), "rig": h.read_rig_poses(n)}


def _assert_identical(got, want, what=""):
    for part in ("pairs", "rig"):
        for k in ("T_rel", "T_abs", "cov", "stats"):
            np.testing.assert_array_equal(got[part][k], want[part][k], err_msg=f"{what} {part}.{k}")


def _ring(h, g, K, P):
    """What BA / loop closure / relocalisation read of frame g: every pair's temporal matches and
    disparities, every left camera's keypoints, level counts and descriptors."""
    slot = h.ring_slot(g)
    out = {"temporal": h.frame_block("temporal", slot, np.int32)[: P * K].copy(),
           "disp": h.frame_block("disp", slot, np.float64)[: P * K].copy()}
    for p in range(P):
        kp = h.keypoints(g, 2 * p)
        for k in ("x", "y", "score", "level", "angle", "counts", "desc"):
            out[f"{p}.{k}"] = np.array(kp[k], copy=True)
    return out


def _run(sc, cfg, sizes, world, transport="copy", max_batch=8, options=None, check=None, rig=True):
    """The unsharded handle and a `world`-rank group fed the same batches; check(b, h1, hs, n)."""
    import torch

    from thor_slam_amd._lib import Handle, HandleGroup

    h1 = Handle(sc["rects"], cfg, max_batch=max_batch)
    hs = [Handle(sc["rects"], cfg, max_batch=max_batch) for _ in range(world)]
    if rig:
        for h in hs + [h1]:
            h.set_rig(sc["E"])
    grp = HandleGroup(hs, transport)
    if options:
        hs[0].shard_options(**options)
    S = sc["frames"].shape[1] // world
    dev = torch.from_numpy(np.ascontiguousarray(sc["frames"])).cuda()
    parts = [dev[:, r * S:(r + 1) * S].contiguous() for r in range(world)]
    s = torch.cuda.current_stream().cuda_stream
    f0 = 0
    try:
        for b, n in enumerate(sizes):
            h1.submit(dev[f0].data_ptr(), n, s)
            grp.submit([p[f0].data_ptr() for p in parts], n)
            check(b, h1, hs, n)
            f0 += n
    finally:
        grp.close()
        for h in hs + [h1]:
            h.close()


@pytest.mark.parametrize("world", [2, 4])
def test_uneven_and_empty_ranges_identical(world):
    """Batches of 3, 8, 1, 2 and 5 frames through max_batch-8 groups (world 4: a 1-frame batch
    leaves three ranks with empty ranges, a 3-frame batch one): every rank's poses equal the
    unsharded handle's, bit for bit."""
    sizes = [3, 8, 1, 2, 5]
    sc = rig_scene(TWO, sum(sizes))

    def check(b, h1, hs, n):
        want = _poses(h1, n)
        for r, h in enumerate(hs):
            _assert_identical(_poses(h, n), want, f"batch {b} ({n} frames) rank {r}")

    _run(sc, HipSlamConfig(), sizes, world, check=check)


def test_rccl_world_one_short_batch():
    """tslam_comm_init at world 1 with batches shorter than max_batch (the RCCL transport's
    all-gather count follows the batch)."""
    import torch

    from thor_slam_amd._lib import Handle, comm_unique_id

    sizes = [3, 8, 1]
    sc = rig_scene(TWO, sum(sizes))
    cfg = HipSlamConfig()
    h1 = Handle(sc["rects"], cfg, max_batch=8)
    h1.set_rig(sc["E"])
    h = Handle(sc["rects"], cfg, max_batch=8)
    h.set_rig(sc["E"])
    h.comm_init(comm_unique_id(), 0, 1)
    dev = torch.from_numpy(np.ascontiguousarray(sc["frames"])).cuda()
    s = torch.cuda.current_stream().cuda_stream
    f0 = 0
    for n in sizes:
        h1.submit(dev[f0].data_ptr(), n, s)
        h.submit_sharded(dev[f0].data_ptr(), n, s)
        _assert_identical(_poses(h, n), _poses(h1, n), f"{n} frames")
        f0 += n
    h.close()
    h1.close()


def test_state_gather_fills_rank0_ring():
    """TSLAM_SHARD_GATHER: after every batch rank 0's ring holds, for every frame of the batch,
    the temporal matches and disparities of every pair and the keypoints / descriptors of every
    left camera, byte for byte as the unsharded handle's ring (4 ranks, one stream each)."""
    sizes = [8, 5, 8]
    sc = rig_scene(TWO, sum(sizes))
    cfg = HipSlamConfig()
    P, K = len(sc["rects"]), cfg.n_features
    seen = {"f0": 0}

    def check(b, h1, hs, n):
        for g in range(seen["f0"], seen["f0"] + n):
            want, got = _ring(h1, g, K, P), _ring(hs[0], g, K, P)
            for k in want:
                np.testing.assert_array_equal(got[k], want[k], err_msg=f"frame {g} {k}")
        seen["f0"] += n

    _run(sc, cfg, sizes, 4, options={"gather": True}, check=check)


def _ba_identical(names, world, sizes, check_every=True):
    cfg = HipSlamConfig(ba_window=10)
    sc = rig_scene(names, sum(sizes), traj_len=max(40, sum(sizes)))
    P = len(sc["rects"])

    def check(b, h1, hs, n):
        _assert_identical(_poses(hs[0], n), _poses(h1, n), f"batch {b}")
        if not check_every and b != len(sizes) - 1:
            return
        for q in [P] + list(range(P)):   # the rig's body window, then every pair's
            want, got = h1.ba_read(q), hs[0].ba_read(q)
            for k in want:
                np.testing.assert_array_equal(got[k], want[k], err_msg=f"batch {b} window {q} {k}")

    _run(sc, cfg, sizes, world, check=check)


def test_local_ba_on_sharded_rig_identical():
    """Local BA on a sharded rig (implied gather): rank 0's rig-level window — body poses, every
    pair's cameras, landmark ids, positions and observations — equals the unsharded handle's after
    every batch, including a short last batch (8 + 8 + 2 frames, 4 ranks)."""
    _ba_identical(TWO, 4, [8, 8, 2])


@pytest.mark.slow
def test_local_ba_c3_eight_ranks_identical():
    """C3 (8 streams, 4 pairs) over 8 ranks with local BA: rank 0's windows == one handle's."""
    _ba_identical(C3_SOURCES, 8, [8, 8, 4], check_every=False)


def test_results_slots_and_profile():
    """TSLAM_SHARD_RESULTS: tslam_poll_batch on every rank returns each batch's poses (as
    tslam_read_poses) in order; TSLAM_SHARD_PROFILE: tslam_shard_timing reports the batch count
    and a positive duration for the kernels and exchanges a rank ran."""
    sizes = [8, 6]
    sc = rig_scene(TWO, sum(sizes))

    def check(b, h1, hs, n):
        want = _poses(h1, n)
        for r, h in enumerate(hs):
            res = h.poll_batch(block=True)
            assert res is not None and res["n"] == n
            np.testing.assert_array_equal(res["T_abs"], want["pairs"]["T_abs"], err_msg=f"rank {r}")
            np.testing.assert_array_equal(res["rig"]["T_abs"], want["rig"]["T_abs"], err_msg=f"rank {r}")
            assert h.poll_batch(block=False) is None
        if b == len(sizes) - 1:
            t, nb = hs[1].shard_timing()
            assert nb == len(sizes)
            for k in ("rectify_pyramid", "detect", "select", "describe", "pack", "import", "match", "match_refine",
                      "pose", "rig", "pose_gather", "chain"):
                assert t[k] > 0.0, (k, t)
            assert t["local_ba"] == 0.0
            assert hs[1].shard_timing()[1] == 0   # reset by the call

    _run(sc, HipSlamConfig(), sizes, 2, options={"results": True, "profile": True}, check=check)


def test_pipelined_batches_identical():
    """TSLAM_SHARD_PIPELINE: the caller's stream waits only for each batch's input, so batch s+1's
    front end runs beside batch s's back end (batches submitted back to back, each polled from the
    result slots one submission later): every batch's poses equal the unsharded handle's."""
    import torch

    from thor_slam_amd._lib import Handle, HandleGroup

    sizes = [8, 8, 3, 8, 5]
    sc = rig_scene(TWO, sum(sizes))
    cfg = HipSlamConfig()
    h1 = Handle(sc["rects"], cfg, max_batch=8)
    h1.set_rig(sc["E"])
    dev = torch.from_numpy(np.ascontiguousarray(sc["frames"])).cuda()
    s = torch.cuda.current_stream().cuda_stream
    want, f0 = [], 0
    for n in sizes:
        h1.submit(dev[f0].data_ptr(), n, s)
        want.append(_poses(h1, n))
        f0 += n
    h1.close()
    world = 4
    hs = [Handle(sc["rects"], cfg, max_batch=8) for _ in range(world)]
    for h in hs:
        h.set_rig(sc["E"])
    grp = HandleGroup(hs, "copy")
    hs[0].shard_options(results=True, pipeline=True)
    S = sc["frames"].shape[1] // world
    parts = [dev[:, r * S:(r + 1) * S].contiguous() for r in range(world)]

    def check(b):
        res = hs[0].poll_batch(block=True)
        assert res is not None and res["n"] == sizes[b]
        np.testing.assert_array_equal(res["T_abs"], want[b]["pairs"]["T_abs"], err_msg=f"batch {b}")
        np.testing.assert_array_equal(res["stats"], want[b]["pairs"]["stats"], err_msg=f"batch {b}")
        np.testing.assert_array_equal(res["rig"]["T_abs"], want[b]["rig"]["T_abs"], err_msg=f"batch {b}")

    try:
        f0 = 0
        for b, n in enumerate(sizes):
            grp.submit([p[f0].data_ptr() for p in parts], n)
            f0 += n
            if b:
                check(b - 1)
        check(len(sizes) - 1)
        torch.cuda.synchronize()
        _assert_identical(_poses(hs[2], sizes[-1]), want[-1], "last batch, rank 2")
    finally:
        grp.close()
        for h in hs:
            h.close()


def test_solo_profiles_rank0_only():
    """TSLAM_SHARD_SOLO (profiling aid): after a full batch, rank 0 alone runs its work with the
    exchanges skipped; its profile counts the solo batches, the other ranks' none."""
    import torch

    from thor_slam_amd._lib import Handle, HandleGroup

    sc = rig_scene(TWO, 16)
    cfg = HipSlamConfig()
    hs = [Handle(sc["rects"], cfg, max_batch=8) for _ in range(4)]
    for h in hs:
        h.set_rig(sc["E"])
    grp = HandleGroup(hs, "copy")
    dev = torch.from_numpy(np.ascontiguousarray(sc["frames"])).cuda()
    parts = [dev[:, r:r + 1].contiguous() for r in range(4)]
    try:
        grp.submit([p[0].data_ptr() for p in parts], 8)
        hs[0].shard_options(solo=True, pipeline=True, profile=True)
        for _ in range(2):
            grp.submit([p[8].data_ptr() for p in parts], 8)
        torch.cuda.synchronize()
        t0, nb0 = hs[0].shard_timing()
        assert nb0 == 2 and t0["detect"] > 0.0 and t0["pose"] > 0.0 and t0["pose_gather"] >= 0.0
        assert hs[1].shard_timing()[1] == 0
    finally:
        grp.close()
        for h in hs:
            h.close()


def _pair_split_identical(names, world, sizes, rig=True, options=None):
    sc = rig_scene(names, sum(sizes))

    def check(b, h1, hs, n):
        import torch

        torch.cuda.synchronize()   # every rank on this device: pipelined batches have finished
        if options and options.get("results"):
            for r, h in enumerate(hs):
                res = h.poll_batch(block=True)
                assert res is not None and res["n"] == n, (b, r)
        want = _poses(h1, n) if rig else {"pairs": h1.read_poses(n)}
        for r, h in enumerate(hs):
            got = _poses(h, n) if rig else {"pairs": h.read_poses(n)}
            for part in want:
                for k in ("T_rel", "T_abs", "cov", "stats"):
                    np.testing.assert_array_equal(got[part][k], want[part][k],
                                                  err_msg=f"batch {b} ({n} frames) rank {r} {part}.{k}")

    _run(sc, HipSlamConfig(), sizes, world, options={"pairs": True, **(options or {})}, check=check, rig=rig)


@pytest.mark.parametrize("names,world,rig", [(TWO[:1], 2, False), (TWO[:1], 2, True), (TWO, 4, True)])
def test_pair_split_identical(names, world, rig):
    """TSLAM_SHARD_PAIRS: rank r solves pair r/2 over half r&1 of each batch from its partner's
    images and stream blocks only, the rig ranges gather the other pairs' pair blocks (pose,
    stats, the 5 correspondence columns the rig pose reads).  Batches of 3, 8, 1, 2, 5 frames
    (uneven and empty halves, frame -1 from the previous batch): every rank's pair and rig poses,
    covariances and statistics equal the unsharded handle's, bit for bit."""
    _pair_split_identical(names, world, [3, 8, 1, 2, 5], rig=rig)


def test_pair_split_pipelined_results_identical():
    """The pair split with TSLAM_SHARD_PIPELINE + TSLAM_SHARD_RESULTS (4 ranks, 2 pairs): batches
    polled from the result slots equal the unsharded handle's."""
    _pair_split_identical(TWO, 4, [8, 8, 3], options={"pipeline": True, "results": True})


@pytest.mark.slow
def test_pair_split_c3_eight_ranks_identical():
    """C3 (4 pairs, 8 streams) over 8 ranks with the pair split: rig poses identical."""
    _pair_split_identical(C3_SOURCES, 8, [8, 5, 8])


def test_pair_split_options_checked():
    """TSLAM_SHARD_PAIRS needs one camera per rank and no state gather / local BA; the profile
    reports the pair-block segment."""
    import torch

    from thor_slam_amd._lib import Handle, HandleGroup

    sc = rig_scene(TWO, 8)
    hs = [Handle(sc["rects"], HipSlamConfig(), max_batch=8) for _ in range(2)]   # 2 cameras per rank
    grp = HandleGroup(hs, "copy")
    try:
        with pytest.raises(RuntimeError, match="one camera per rank"):
            hs[0].shard_options(pairs=True)
    finally:
        grp.close()
        for h in hs:
            h.close()
    hs = [Handle(sc["rects"], HipSlamConfig(ba_window=10), max_batch=8) for _ in range(4)]
    grp = HandleGroup(hs, "copy")
    try:
        with pytest.raises(RuntimeError, match="without the state gather"):
            hs[0].shard_options(pairs=True)
    finally:
        grp.close()
        for h in hs:
            h.close()
    hs = [Handle(sc["rects"], HipSlamConfig(), max_batch=8) for _ in range(4)]
    for h in hs:
        h.set_rig(sc["E"])
    grp = HandleGroup(hs, "copy")
    dev = torch.from_numpy(np.ascontiguousarray(sc["frames"])).cuda()
    parts = [dev[:, r:r + 1].contiguous() for r in range(4)]
    try:
        hs[0].shard_options(pairs=True, profile=True)
        grp.submit([p[0].data_ptr() for p in parts], 8)
        torch.cuda.synchronize()
        for r in range(4):
            t, nb = hs[r].shard_timing()
            assert nb == 1 and t["pair_blocks"] > 0.0 and t["rig"] > 0.0 and t["import"] > 0.0, (r, t)
    finally:
        grp.close()
        for h in hs:
            h.close()
