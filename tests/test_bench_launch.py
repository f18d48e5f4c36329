"""bench.py's self-launch of N ranks (``python bench.py --gpus N`` without a torch.distributed
wrapper): the command, the environment each rank sees, rank 0's line on stdout, and the timeout
that keeps a stuck rank from hanging the job.  CPU only (gloo)."""

from __future__ import annotations

import json
import sys
import textwrap
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402


def test_launch_command_shape():
    cmd = bench.launch_command(4, ["--gpus", "4", "--steps", "3"], 29555)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert "--master-port=29555" in cmd
    assert cmd[-4:] == [str(ROOT / "bench.py"), "--gpus", "4", "--steps", "3"][-4:]
    assert cmd[-5] == str(ROOT / "bench.py")


RANK_SCRIPT = textwrap.dedent("""
    import json, os, sys
    import torch.distributed as dist
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    assert os.environ["MASTER_ADDR"] == "127.0.0.1"
    dist.init_process_group("gloo")
    import torch
    t = torch.tensor([float(rank + 1)])
    dist.all_reduce(t)
    dist.barrier()
    if rank == 0:
        print(json.dumps({"world": world, "sum": float(t.item()), "argv": sys.argv[1:],
                          "ipc": os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY")}), flush=True)
    dist.destroy_process_group()
""")


def test_self_launch_runs_ranks_and_prints_rank0(tmp_path, capfd, monkeypatch):
    script = tmp_path / "rank.py"
    script.write_text(RANK_SCRIPT)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("WORLD_SIZE_UNRELATED", "x")
    rc = bench.self_launch(2, ["--gpus", "2", "--dist-backend", "gloo"], 120, script=script)
    out = capfd.readouterr().out
    assert rc == 0, out
    lines = [json.loads(l) for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out        # rank 0 only
    assert lines[0]["world"] == 2 and lines[0]["sum"] == 3.0
    assert lines[0]["argv"] == ["--gpus", "2", "--dist-backend", "gloo"]
    assert lines[0]["ipc"] == "0"


def test_self_launch_failure_and_timeout_exit_nonzero(tmp_path):
    bad = tmp_path / "bad.py"
    bad.write_text("import os, sys\nsys.exit(3 if os.environ['RANK'] == '1' else 0)\n")
    assert bench.self_launch(2, [], 120, script=bad) != 0
    hang = tmp_path / "hang.py"
    hang.write_text("import time\ntime.sleep(600)\n")
    assert bench.self_launch(2, [], 5, script=hang) == 124
