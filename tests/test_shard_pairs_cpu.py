"""The pair-split layout of the sharded stereo rig (TSLAM_SHARD_PAIRS, csrc/tslam_shard.cpp) on CPU.

Four ranks over gloo, one camera each (two stereo sources), the NumPy oracle as each rank's
compute, the layout's own routing:
* rank r extracts features of camera r for every frame of the batch;
* its partner r ^ 1 sends it the raw frames lo - 1 .. hi - 1 of its half (peer_range(r & 1, n, 2));
* rank r solves pair r // 2 (stereo, temporal, pose) over that half alone;
* pair blocks — status, T, cov and the five correspondence columns the rig pose reads (X, Y, Z, du,
  dv) — go to the ranks of the same half, for each one's rig range: range rig_slot(r) =
  (r & 1) * world / 2 + r // 2 of the world-way split, which lies inside r's half;
* each rank solves the rig pose of its rig range, the pose rows are all-gathered in rig-slot order
  and every rank chains the batch.
Every rank must reproduce the sequential oracle (per-pair trackers + oracle/numpy_rig.py) exactly,
as tests/test_shard_cpu.py does for the frame-range layout."""

from __future__ import annotations

import os

import numpy as np
import torch.multiprocessing as mp

from test_shard_cpu import BATCH, NB, _cfg, _chain, _features, _free_port, _rect_dict, _rig

WORLD = 4
PAIR_COLS = ("X", "Y", "Z", "du", "dv")   # the columns of a correspondence the rig pose reads


def _peer_range(q: int, n: int, world: int) -> tuple[int, int]:   # tslam_ranges.h
    return q * n // world, (q + 1) * n // world


def _rig_slot(r: int, world: int) -> int:
    return (r & 1) * (world // 2) + (r >> 1)


def _pair_back_end(feats, rect, p, cfg, g0, lo, hi):
    """Oracle A6/A7 of pair p for batch frames [lo, hi) from its features of frames lo-1 .. hi-1:
    per frame (status, T, cov, corr restricted to PAIR_COLS)."""
    from oracle import numpy_slam as O

    disp = {}
    for g in range(g0 + lo - 1, g0 + hi):
        if g >= 0:
            fl, fr = feats[(g, 2 * p)], feats[(g, 2 * p + 1)]
            sm = O.match(fl, fr, cfg, "stereo")
            disp[g] = O.stereo_subpixel(fl, fr, sm[0], fl["levels"], fr["levels"])
    out = {}
    intr = (rect.fx, rect.fy, rect.cx, rect.cy)
    for f in range(lo, hi):
        g = g0 + f
        if g == 0:
            out[f] = (2, np.eye(4), np.zeros((6, 6)), None)
            continue
        cur, prev = feats[(g, 2 * p)], feats[(g - 1, 2 * p)]
        tm = O.match(cur, prev, cfg, "temporal")
        corr = O.build_correspondences({"left": prev, "disp": disp[g - 1]}, {"left": cur}, tm[0],
                                       intr + (rect.fx * rect.baseline,))
        est = O.estimate_pose(corr, intr, cfg, g)
        out[f] = (est["status"], est["T"], est["cov"], {k: np.asarray(corr[k]).copy() for k in PAIR_COLS})
    return out


def _worker(rank, world, port, out_dir):
    import torch
    import torch.distributed as dist

    from oracle.numpy_rig import rig_pose

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg, sc = _cfg(), _rig()
    rects, E, frames = sc["rects"], sc["E"], sc["frames"]
    P = len(rects)
    assert 2 * P == world
    p, partner = rank // 2, rank ^ 1
    H, W = frames.shape[2:]
    feats, state = {}, [np.eye(4) for _ in range(P + 1)]
    prev_raw = np.zeros((H, W), np.uint8)
    lo, hi = _peer_range(rank & 1, BATCH, 2)            # this rank's half of the batch
    plo, phi = _peer_range(partner & 1, BATCH, 2)       # the partner's
    rlo, rhi = _peer_range(_rig_slot(rank, world), BATCH, world)
    assert lo <= rlo and rhi <= hi                      # the rig range nests in the half
    per = BATCH // 2 + 1
    rows_out, abs_out = [], []
    for b in range(NB):
        g0 = b * BATCH
        mine = frames[g0:g0 + BATCH, rank]              # this rank's camera
        for f in range(BATCH):
            feats[(g0 + f, rank)] = _features(mine[f], rects[p], rank % 2, cfg)
        # raw frames plo-1 .. phi-1 of my camera to the partner (frame -1: the previous batch's last)
        send = np.zeros((per, H, W), np.uint8)
        for k, f in enumerate(range(plo - 1, phi)):
            send[k] = prev_raw if f < 0 else mine[f]
        prev_raw = mine[-1].copy()
        recv = torch.empty((per, H, W), dtype=torch.uint8)
        reqs = [dist.isend(torch.from_numpy(send), partner), dist.irecv(recv, partner)]
        for rq in reqs:
            rq.wait()
        for k, f in enumerate(range(lo - 1, hi)):
            if g0 + f >= 0:
                feats[(g0 + f, partner)] = _features(recv[k].numpy(), rects[p], partner % 2, cfg)
        mine_pair = _pair_back_end(feats, rects[p], p, cfg, g0, lo, hi)
        # pair blocks: my pair's frames of each same-half rank's rig range (everyone's, gathered)
        blocks = [None] * world
        dist.all_gather_object(blocks, {f: mine_pair[f] for f in range(lo, hi)})
        rows = np.zeros((rhi - rlo, P + 1, 53))
        for f in range(rlo, rhi):
            g = g0 + f
            items = []
            for q in range(P):
                src = 2 * q + (rank & 1)                # the rank of pair q's half that holds frame f
                st, T, cov, corr = blocks[src][f]
                items.append({"status": st, "T": T, "corr": corr, "intr": (rects[q].fx, rects[q].fy, rects[q].cx, rects[q].cy)})
                rows[f - rlo, q] = np.concatenate([T.ravel(), cov.ravel(), [st]])
            rig = {"T": np.eye(4), "cov": np.zeros((6, 6)), "status": 2} if g == 0 else rig_pose(items, E, cfg)
            rows[f - rlo, P] = np.concatenate([rig["T"].ravel(), rig["cov"].ravel(), [rig["status"]]])
        every = [None] * world
        dist.all_gather_object(every, rows)
        by_slot = [None] * world
        for q in range(world):
            by_slot[_rig_slot(q, world)] = every[q]
        rows_all = np.concatenate(by_slot)
        assert rows_all.shape[0] == BATCH
        rows_out.append(rows_all)
        abs_out.append(_chain(rows_all, state))
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), rows=np.stack(rows_out), t_abs=np.stack(abs_out))
    dist.barrier()
    dist.destroy_process_group()


def test_pair_split_decomposition_matches_sequential_oracle(tmp_path):
    from oracle import numpy_slam as O
    from oracle.numpy_rig import RigChain, rig_pose

    mp.spawn(_worker, args=(WORLD, _free_port(), str(tmp_path)), nprocs=WORLD, join=True)
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
    for r in range(WORLD):
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
                assert rows[b, f, -1, 52] == st, (r, b, f)
                np.testing.assert_array_equal(rows[b, f, -1, :16].reshape(4, 4), T)
                np.testing.assert_allclose(t_abs[b, f, -1].reshape(4, 4), T_abs, rtol=0, atol=1e-12)
