"""One rank of tests/test_gpu_shard.py's DistShardedRig tests (launched by torch.distributed.run):
the 2-pair bracket rig sharded over WORLD_SIZE processes with DistShardedRig on the gloo backend
(host-staged) or the nccl (RCCL) backend; writes its per-batch poses to <out>/rank<r>.json.

With a fifth argument ``rgbd`` the rig is the 4-camera RGB-D rig (one camera per rank at world 4,
pair-block exchange) at 640x400.

usage: shard_worker.py OUT BATCH NB [gloo|nccl] [rgbd]"""

from __future__ import annotations

import json
import sys
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist

from helpers import rgbd_rig_scene, rig_scene
from thor_slam_amd.params import HipSlamConfig
from thor_slam_amd.shard import DistShardedRig


def main() -> None:
    out, batch, nb = Path(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    backend = sys.argv[4] if len(sys.argv) > 4 else "gloo"
    torch.cuda.set_device(0)
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    rgbd = len(sys.argv) > 5 and sys.argv[5] == "rgbd"
    if rgbd:
        sc = rgbd_rig_scene(n=batch * nb, width=640, height=400)
        frames = sc["records"]
    else:
        sc = rig_scene(("192.168.2.21", "192.168.2.25"), batch * nb)
        frames = sc["frames"]
    rig = DistShardedRig(sc["rects"], HipSlamConfig(rgbd=rgbd), batch, base_T_rect=sc["E"])
    S = rig.plan.streams_per_rank
    mine = torch.from_numpy(np.ascontiguousarray(frames[:, rank * S:(rank + 1) * S])).cuda()
    res = []
    for b in range(nb):
        rig.step(mine[b * batch:(b + 1) * batch])
        r = rig.read()
        res.append({part: {k: np.asarray(v).tolist() for k, v in r[part].items() if k != "cov"} for part in r})
    rig.close()
    (out / f"rank{rank}.json").write_text(json.dumps(res))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
