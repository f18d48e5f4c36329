"""The sharded rig's decomposition on CPU (thor_slam_amd/shard.py).

The device path shards a rig's cameras (front end) and a batch's frames (back end) over ranks,
routes raw images with an all-to-all and pose records with an all-gather, and chains every batch
on every rank.  Here the same ShardPlan and the same routing run over gloo with world_size 2,
with the NumPy oracle as each rank's compute: each rank extracts features for its own cameras,
receives the raw frames lo-1 .. hi-1 of the others (byte layout of RankShard.stage_raw), runs
stereo for lo-1 .. hi-1 and temporal + pose + rig pose for lo .. hi-1, all-gathers the f64 pose
records and chains.  Both ranks must reproduce the sequential oracle (per-pair trackers +
oracle/numpy_rig.py) exactly.
"""

from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from thor_slam_amd.shard import ShardPlan

BATCH, NB, W, H = 4, 2, 320, 200
NAMES = ("192.168.2.21", "192.168.2.25")


def _cfg():
    from thor_slam_amd.params import HipSlamConfig

    return HipSlamConfig(n_features=400, n_levels=2)


def test_plan_ranges():
    p = ShardPlan(n_cams=8, world=8, batch=256)
    assert p.streams_per_rank == 1 and p.frames_per_rank == 32 and p.recv_frames == 33
    assert p.cams(3) == (3, 4) and p.frames(3) == (96, 128) and p.sent_frames(0) == (-1, 32)
    p = ShardPlan(n_cams=8, world=2, batch=256)
    assert p.cams(1) == (4, 8) and p.frames(1) == (128, 256)
    covered = sorted(f for r in range(8) for f in range(*ShardPlan(8, 8, 64).frames(r)))
    assert covered == list(range(64))
    with pytest.raises(ValueError):
        ShardPlan(n_cams=8, world=3, batch=255)
    with pytest.raises(ValueError):
        ShardPlan(n_cams=8, world=4, batch=250)


def _rig():
    from helpers import rig_scene

    return rig_scene(NAMES, BATCH * NB, width=W, height=H)


def _rect_dict(r):
    return dict(fx=r.fx, fy=r.fy, cx=r.cx, cy=r.cy, baseline=r.baseline, map_l=r.map_left, map_r=r.map_right)


def _features(img, rect, side, cfg):
    from oracle import numpy_slam as O

    return O.extract(O.remap(img, rect.map_left if side == 0 else rect.map_right), cfg)


def _back_end(feats, rects, E, cfg, g0, lo, hi):
    """Oracle A6/A7 + rig pose for batch frames [lo, hi) from features of frames lo-1 .. hi-1:
    rows [P+1][T(16) | cov(36) | status] (the pairs, then the rig)."""
    from oracle import numpy_slam as O
    from oracle.numpy_rig import rig_pose

    P = len(rects)
    disp = {}
    for g in range(g0 + lo - 1, g0 + hi):
        if g < 0:
            continue
        for p in range(P):
            fl, fr = feats[(g, 2 * p)], feats[(g, 2 * p + 1)]
            sm = O.match(fl, fr, cfg, "stereo")
            disp[(g, p)] = O.stereo_subpixel(fl, fr, sm[0], fl["levels"], fr["levels"])
    rows = np.zeros((hi - lo, P + 1, 53))
    for f in range(lo, hi):
        g = g0 + f
        items = []
        for p, r in enumerate(rects):
            intr = (r.fx, r.fy, r.cx, r.cy)
            if g == 0:
                est = {"T": np.eye(4), "cov": np.zeros((6, 6)), "status": 2, "corr": None}
            else:
                cur, prev = feats[(g, 2 * p)], feats[(g - 1, 2 * p)]
                tm = O.match(cur, prev, cfg, "temporal")
                corr = O.build_correspondences({"left": prev, "disp": disp[(g - 1, p)]}, {"left": cur}, tm[0],
                                               intr + (r.fx * r.baseline,))
                est = O.estimate_pose(corr, intr, cfg, g)
                est["corr"] = corr
            items.append({"status": est["status"], "T": est["T"], "corr": est["corr"], "intr": intr})
            rows[f - lo, p] = np.concatenate([est["T"].ravel(), est["cov"].ravel(), [est["status"]]])
        rig = {"T": np.eye(4), "cov": np.zeros((6, 6)), "status": 2} if g == 0 else rig_pose(items, E, cfg)
        rows[f - lo, P] = np.concatenate([rig["T"].ravel(), rig["cov"].ravel(), [rig["status"]]])
    return rows


def _chain(rows_all, state):
    """Per-pair and rig chaining of one batch (k_chain's rule): T_abs = T_abs inv(T_rel) on success."""
    out = np.zeros(rows_all.shape[:2] + (16,))
    for f in range(rows_all.shape[0]):
        for q in range(rows_all.shape[1]):
            T = rows_all[f, q, :16].reshape(4, 4)
            if rows_all[f, q, 52] == 0:
                inv = np.eye(4)
                inv[:3, :3] = T[:3, :3].T
                inv[:3, 3] = -(T[:3, :3].T @ T[:3, 3])
                state[q] = state[q] @ inv
            out[f, q] = state[q].ravel()
    return out


def _worker(rank, world, port, out_dir):
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg, sc = _cfg(), _rig()
    rects, E, frames = sc["rects"], sc["E"], sc["frames"]
    P, C = len(rects), 2 * len(rects)
    plan = ShardPlan(C, world, BATCH)
    S = plan.streams_per_rank
    c0, c1 = plan.cams(rank)
    lo, hi = plan.frames(rank)
    feats, state = {}, [np.eye(4) for _ in range(P + 1)]
    prev_raw = np.zeros((S, H, W), np.uint8)
    rows_out, abs_out = [], []
    for b in range(NB):
        g0 = b * BATCH
        mine = frames[g0:g0 + BATCH, c0:c1]                       # this rank's streams
        for f in range(BATCH):                                     # front end of its cameras
            for c in range(c0, c1):
                feats[(g0 + f, c)] = _features(mine[f, c - c0], rects[c // 2], c % 2, cfg)
        send = np.zeros((world, plan.recv_frames, S, H, W), np.uint8)   # RankShard.stage_raw layout
        for q in range(world):
            a, z = plan.sent_frames(q)
            send[q, 0] = prev_raw if a < 0 else mine[a]
            send[q, 1:] = mine[a + 1:z]
        prev_raw = mine[-1].copy()
        recv = torch.empty(send.shape, dtype=torch.uint8)
        dist.all_to_all_single(recv, torch.from_numpy(send))
        recv = recv.numpy()
        for q in range(world):                                     # the other ranks' cameras, frames lo-1 .. hi-1
            if q == rank:
                continue
            q0, q1 = plan.cams(q)
            for k in range(plan.recv_frames):
                g = g0 + lo - 1 + k
                if g < 0:
                    continue
                for c in range(q0, q1):
                    feats[(g, c)] = _features(recv[q, k, c - q0], rects[c // 2], c % 2, cfg)
        rows = _back_end(feats, rects, E, cfg, g0, lo, hi)
        every = torch.empty((world * rows.shape[0],) + rows.shape[1:], dtype=torch.float64)
        dist.all_gather_into_tensor(every, torch.from_numpy(np.ascontiguousarray(rows)))
        rows_all = every.numpy().reshape((BATCH,) + rows.shape[1:])
        rows_out.append(rows_all)
        abs_out.append(_chain(rows_all, state))
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), rows=np.stack(rows_out), t_abs=np.stack(abs_out))
    dist.barrier()
    dist.destroy_process_group()


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_sharded_decomposition_matches_sequential_oracle(tmp_path):
    from oracle import numpy_slam as O
    from oracle.numpy_rig import RigChain, rig_pose

    mp.spawn(_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    cfg, sc = _cfg(), _rig()
    rects, E, frames = sc["rects"], sc["E"], sc["frames"]
    trks = [O.OracleTracker(cfg, _rect_dict(r)) for r in rects]
    chain = RigChain()
    want_rig, want_pair = [], []
    for i in range(BATCH * NB):
        outs = [trk.step(frames[i, 2 * q], frames[i, 2 * q + 1]) for q, trk in enumerate(trks)]
        want_pair.append([(o["status"], o["T"], o["world_T_cam"]) for o in outs])
        if i == 0:
            want_rig.append((2, np.eye(4), np.eye(4)))
            continue
        items = [{"status": o["status"], "T": o["T"], "corr": o.get("corr"), "intr": (r.fx, r.fy, r.cx, r.cy)}
                 for o, r in zip(outs, rects)]
        res = rig_pose(items, E, cfg)
        want_rig.append((res["status"], res["T"], chain.step(res)))
    assert sum(w[0] == 0 for w in want_rig) >= BATCH * NB - 2   # the rig tracks
    for r in range(2):
        got = np.load(tmp_path / f"rank{r}.npz")
        rows, t_abs = got["rows"], got["t_abs"]
        for b in range(NB):
            for f in range(BATCH):
                i = b * BATCH + f
                for p in range(len(rects)):
                    st, T, wTc = want_pair[i][p]
                    assert rows[b, f, p, 52] == st
                    np.testing.assert_array_equal(rows[b, f, p, :16].reshape(4, 4), T)
                    np.testing.assert_allclose(t_abs[b, f, p].reshape(4, 4), wTc, rtol=0, atol=1e-12)
                st, T, T_abs = want_rig[i]
                assert rows[b, f, -1, 52] == st
                np.testing.assert_array_equal(rows[b, f, -1, :16].reshape(4, 4), T)
                np.testing.assert_allclose(t_abs[b, f, -1].reshape(4, 4), T_abs, rtol=0, atol=1e-12)


def test_sharded_config_validation():
    """HipSlamConfig(devices=...): local BA and batches of any length are allowed on a sharded rig
    (rank 0 solves the window after the state gather; ranges may be uneven), so is the dense map of
    an RGB-D rig (the TSDF lives on rank 0, whose camera is pair 0), and the transport is checked."""
    import pytest

    from thor_slam_amd.params import HipSlamConfig

    HipSlamConfig(devices=(0, 1, 2, 3), ba_window=10, batch_size=6).validate()
    HipSlamConfig(devices=(0, 1), enable_loop_closure=True, batch_size=1).validate()
    HipSlamConfig(devices=(0, 1), rgbd=True, dense_map=True).validate()
    with pytest.raises(ValueError, match="without local BA"):
        HipSlamConfig(devices=(0, 1), rgbd=True, ba_window=4).validate()
    with pytest.raises(ValueError, match="shard_transport"):
        HipSlamConfig(devices=(0, 1), shard_transport="tcp").validate()
