"""C5 (BASELINE.json configs[4]): the 4-camera RGB-D rig (nvblox-shaped, 1280x720 BGR + aligned
u16 depth; scripts/run_pipeline.py:218-256, luxonis.py:876-919) on the brackets.urdf joints.

* one handle for the whole rig vs the oracle (per-camera ``OracleTracker.step_rgbd`` + the rig
  pose of ``oracle/numpy_rig.py``): per-camera results bit-exact / 1e-9 as the single-camera
  RGB-D tests, the rig's status, winning candidate and inlier count identical, body motion and
  chained world_T_base within 1e-9;
* one camera per rank (camera-sharded RGB-D: every rank tracks its own camera over the whole
  batch, pair blocks all-to-all, rig pose per frame range): bit-identical to the one handle, in
  one process (``LocalShardedRig``), through the library's own driver (``tslam_group_*``, copy
  transport; RCCL clique on one device) and with 2 real processes (gloo).
"""

from __future__ import annotations

import functools
import json
import os
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

from helpers import rel_frobenius, rgbd_rig_scene
from oracle import numpy_slam as O
from oracle.numpy_rig import RigChain, rig_pose
from thor_slam_amd.params import HipSlamConfig

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]


@functools.lru_cache(maxsize=1)
def oracle_run(n: int = 5):
    sc = rgbd_rig_scene(n=n)
    cfg = HipSlamConfig(rgbd=True)
    trks = [O.OracleTracker(cfg, dict(fx=r.fx, fy=r.fy, cx=r.cx, cy=r.cy, baseline=r.baseline, map_l=r.map_left,
                                      map_r=r.map_right)) for r in sc["rects"]]
    chain = RigChain()
    per, rig = [], []
    for i in range(n):
        outs = [trk.step_rgbd(*sc["raw"][i][q]) for q, trk in enumerate(trks)]
        per.append(outs)
        if i == 0:
            rig.append({"status": 2, "T_abs": np.eye(4)})
            continue
        items = [{"status": o["status"], "T": o["T"], "corr": o.get("corr"), "intr": (r.fx, r.fy, r.cx, r.cy)}
                 for o, r in zip(outs, sc["rects"])]
        res = rig_pose(items, sc["E"], cfg)
        res["T_abs"] = chain.step(res)
        rig.append(res)
    return sc, cfg, per, rig


def single_handle(sc, cfg, batch, n):
    import torch

    from thor_slam_amd._lib import Handle

    h = Handle(sc["rects"], cfg, max_batch=batch)
    h.set_rig(sc["E"])
    dev = torch.from_numpy(np.ascontiguousarray(sc["records"][:n])).cuda()
    out = []
    for b0 in range(0, n, batch):
        h.submit(dev[b0].data_ptr(), batch, torch.cuda.current_stream().cuda_stream)
        out.append({"pairs": h.read_poses(batch), "rig": h.read_rig_poses(batch)})
    h.close()
    return out


def test_c5_four_camera_rgbd_rig_matches_oracle():
    n = 5
    sc, cfg, per, rig = oracle_run(n)
    got = single_handle(sc, cfg, n, n)[0]
    P = len(sc["rects"])
    assert P == 4 and sc["records"].shape[2] == 5 * 1280 * 720
    for i in range(n):
        for q in range(P):
            o, st = per[i][q], got["pairs"]["stats"][i, q]
            assert st[0] == o["status"], (i, q)
            if i:
                assert st[2] == o["n_inliers"] and st[4] == o["best_hyp"], (i, q)
                assert rel_frobenius(got["pairs"]["T_abs"][i, q], o["world_T_cam"]) < 1e-9, (i, q)
        g, w = got["rig"], rig[i]
        assert g["stats"][i, 0] == w["status"], i
        if i == 0:
            continue
        assert g["stats"][i, 4] == w["best"] and g["stats"][i, 2] == w["n_inliers"], (i, g["stats"][i], w["n_inliers"])
        assert rel_frobenius(g["T_rel"][i], w["T"]) < 1e-9, i
        assert rel_frobenius(g["T_abs"][i], w["T_abs"]) < 1e-9, i
        assert rel_frobenius(g["cov"][i], w["cov"]) < 1e-6, i
    assert (got["rig"]["stats"][1:, 0] == 0).all()
    gt = np.linalg.inv(sc["traj"][0]) @ sc["traj"][n - 1]
    assert np.linalg.norm(got["rig"]["T_abs"][n - 1][:3, 3] - gt[:3, 3]) < 0.05 * np.linalg.norm(gt[:3, 3]) + 2e-3


def assert_identical(got, want):
    for part in ("pairs", "rig"):
        for k in ("T_rel", "T_abs", "cov", "stats"):
            np.testing.assert_array_equal(got[part][k], want[part][k], err_msg=f"{part}.{k}")


@pytest.mark.parametrize("world", [4, 2])
def test_rgbd_rig_one_camera_per_rank_identical(world):
    """LocalShardedRig (all ranks in one process): pair-block all-to-all + rig pose per frame range."""
    import torch

    from thor_slam_amd.shard import LocalShardedRig

    batch, nb = 4, 2
    sc = rgbd_rig_scene(n=batch * nb)
    cfg = HipSlamConfig(rgbd=True)
    want = single_handle(sc, cfg, batch, batch * nb)
    rig = LocalShardedRig(sc["rects"], cfg, world=world, batch=batch, base_T_rect=sc["E"])
    dev = torch.from_numpy(np.ascontiguousarray(sc["records"])).cuda()
    for b in range(nb):
        rig.step(dev[b * batch:(b + 1) * batch])
        for r in range(world):
            assert_identical(rig.read(r), want[b])
    assert (want[-1]["rig"]["stats"][:, 0] == 0).all()
    rig.close()


def _group_run(sc, cfg, frames, world, batch, nb, transport):
    """The library's own driver (tslam_group_*) over `world` handles on this device."""
    import torch

    from thor_slam_amd._lib import Handle, HandleGroup

    hs = [Handle(sc["rects"], cfg, max_batch=batch) for _ in range(world)]
    for h in hs:
        h.set_rig(sc["E"])
    grp = HandleGroup(hs, transport)
    S = frames.shape[1] // world
    parts = [torch.from_numpy(np.ascontiguousarray(frames[:, r * S:(r + 1) * S])).cuda() for r in range(world)]
    out = []
    for b in range(nb):
        grp.submit([p[b * batch].data_ptr() for p in parts])
        out.append([{"pairs": h.read_poses(batch), "rig": h.read_rig_poses(batch)} for h in hs])
    grp.close()
    for h in hs:
        h.close()
    return out


@pytest.mark.parametrize("world", [4, 2])
def test_rgbd_rig_library_driver_identical(world):
    """tslam_group_create(COPY) + tslam_group_submit: the C driver's pair-block packing, exchange
    ordering and double buffering on `world` ranks sharing this GPU, == the one handle."""
    batch, nb = 4, 3
    sc = rgbd_rig_scene(n=batch * nb)
    cfg = HipSlamConfig(rgbd=True)
    want = single_handle(sc, cfg, batch, batch * nb)
    got = _group_run(sc, cfg, sc["records"], world, batch, nb, "copy")
    for b in range(nb):
        for r in range(world):
            assert_identical(got[b][r], want[b])


def test_rgbd_rig_dist_gloo_two_processes(tmp_path):
    """DistShardedRig (torch.distributed, gloo) with 2 processes, 2 RGB-D cameras per rank."""
    batch, nb = 4, 2
    sc = rgbd_rig_scene(n=batch * nb, width=640, height=400)
    want = single_handle(sc, HipSlamConfig(rgbd=True), batch, batch * nb)
    env = dict(os.environ, PYTHONPATH=f"{ROOT}:{ROOT / 'thor-slam_amd'}:{ROOT / 'tests'}")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr=127.0.0.1",
           "--master-port=29527", str(ROOT / "tests" / "shard_worker.py"), str(tmp_path), str(batch), str(nb), "gloo",
           "rgbd"]
    subprocess.run(cmd, check=True, env=env, timeout=240)
    for r in range(2):
        got = json.loads((tmp_path / f"rank{r}.json").read_text())
        for b in range(nb):
            for part in ("pairs", "rig"):
                for k in ("T_rel", "T_abs", "stats"):
                    np.testing.assert_array_equal(np.array(got[b][part][k]), want[b][part][k], err_msg=f"{r} {b} {part}.{k}")
