"""GPU: the sharded step over RCCL (torch.distributed "nccl" backend) -- tools/rccl_smoke.py in a
child process (its own process group, world size 1: the RCCL world a one-GPU box has; the
multi-GPU bench runs the same code at N = 2..8): dist.all_reduce of the shared gradient block wired
into PertShard gives losses bit-identical to the unsharded step."""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_sharded_step_over_rccl_matches_unsharded():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "rccl_smoke.py")], env=env, cwd=ROOT,
                         capture_output=True, text=True, timeout=180)
    print(out.stdout[-2000:])
    assert out.returncode == 0, out.stderr[-3000:]
    assert "rccl smoke ok" in out.stdout
