"""RCCL on the product's sharded path, one GPU (world size 1 -- the only RCCL world a one-GPU
box has; the driver's multi-GPU bench runs the same path at N = 2..8):

* ``torch.distributed`` over the "nccl" backend (RCCL) initialised as bench.py does it;
* the shard's step with the all-reduce wired in (PertShard(allreduce=...): finalize into
  grad_local, copy, ``dist.all_reduce`` of the shared block, Adam) against the same shard
  without it -- identical losses (a world-size-1 sum is the identity);
* the per-step cost of the RCCL call at the shared block's size (44 KB fp64 at 5,451 bins).

usage: python tools/rccl_smoke.py   (sets RANK / WORLD_SIZE / MASTER_* itself)
"""
import os
import sys
import time

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29533")
os.environ.setdefault("RANK", "0")
os.environ.setdefault("WORLD_SIZE", "1")

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from scdna_replication_tools_amd.engine import PertShard
    from tests._problems import KIND_OF, init_constrained, make_problem
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    t = torch.arange(5452, dtype=torch.float64, device=dev)
    dist.all_reduce(t)
    torch.cuda.synchronize()
    assert torch.equal(t, torch.arange(5452, dtype=torch.float64, device=dev))
    n = 200
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        dist.all_reduce(t)
    torch.cuda.synchronize()
    print("RCCL all_reduce of {} fp64 (world 1): {:.1f} us per call".format(t.numel(), (time.perf_counter() - t0) / n * 1e6),
          flush=True)

    def allreduce(x):
        dist.all_reduce(x, op=dist.ReduceOp.SUM)

    prob, kw, z = make_problem("step2", L=600, N=300, seed=3)
    losses = {}
    for name, ar in (("plain", None), ("rccl", allreduce)):
        sh = PertShard(KIND_OF["step2"], init=init_constrained("step2", z), device=dev, allreduce=ar, **kw)
        sh.set_unconstrained({k: v.numpy() for k, v in z.items()})
        losses[name], _ = sh.run_svi(40, 10 ** 9, 0.0)
    a, b = np.asarray(losses["plain"]), np.asarray(losses["rccl"])
    print("sharded path over RCCL vs unsharded: 40 steps, max |dloss| / |loss| = {:.2e}".format(
        float(np.abs(a - b).max() / np.abs(a).max())), flush=True)
    assert np.array_equal(a, b), (a[:3], b[:3])
    dist.destroy_process_group()
    print("rccl smoke ok", flush=True)


if __name__ == "__main__":
    main()
