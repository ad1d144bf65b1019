"""World-size-2 gloo test of the cell-sharded decomposition (CPU, no GPU).

Each rank evaluates the oracle on its contiguous cell shard, with the global priors
on rank 0 only (what ``is_root`` does on the device), and all-reduces the shared-site
gradients and the loss with ``sharding.make_allreduce`` -- the same call PertShard makes.
The result must equal the single-process full-problem loss and gradients.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from scdna_replication_tools_amd.sharding import cell_bounds, make_allreduce, shard_slice


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, kind, out_path):
    from oracle import pert_oracle as po
    from tests._problems import make_problem
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:{}".format(port), rank=rank, world_size=world)
    try:
        prob, _, z = make_problem(kind, L=12, N=9, seed=21)
        sl = shard_slice(9, world, rank)
        sub = prob.cells(sl)
        zz = {}
        for name, _ in po.PARAM_SITES[kind]:
            v = z[name].detach().clone()
            if name in ("expose_tau", "expose_u", "expose_betas"):
                v = v[sl]
            elif name == "expose_pi":
                v = v[:, sl]
            zz[name] = v.requires_grad_(True)
        c = po.constrain(kind, zz)
        ploidy = po.cell_ploidies(prob)[sl]
        loss = -sum(po.model_terms(sub, c, global_terms=(rank == 0), ploidy=ploidy).values())
        loss.backward()
        shared = [n for n in ("expose_rho", "expose_a", "expose_lambda", "expose_beta_stds", "expose_beta_means")
                  if n in zz]
        buf = torch.cat([zz[n].grad.reshape(-1) for n in shared] + [loss.detach().reshape(1)]).double()
        ar = make_allreduce()
        assert ar is not None
        ar(buf)
        if rank == 0:
            torch.save({"buf": buf, "shared": shared, "tau_grad0": zz["expose_tau"].grad.clone()}, out_path)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("kind", ["step2", "step1"])
def test_two_rank_decomposition_matches_full(tmp_path, kind):
    from oracle import pert_oracle as po
    from tests._problems import make_problem
    out = str(tmp_path / "r0.pt")
    mp.spawn(_worker, args=(2, _free_port(), kind, out), nprocs=2, join=True)
    got = torch.load(out, weights_only=True)
    prob, _, z = make_problem(kind, L=12, N=9, seed=21)
    loss, g = po.loss_and_grads(prob, z)
    want = torch.cat([g[n].reshape(-1) for n in got["shared"]] + [loss.reshape(1)]).double()
    torch.testing.assert_close(got["buf"], want, rtol=1e-10, atol=1e-8)
    torch.testing.assert_close(got["tau_grad0"], g["expose_tau"][shard_slice(9, 2, 0)], rtol=1e-10, atol=1e-10)


def test_cell_bounds_balanced():
    b = cell_bounds(10000, 8)
    sizes = [e - s for s, e in b]
    assert sum(sizes) == 10000 and max(sizes) - min(sizes) <= 1
    assert b[0][0] == 0 and b[-1][1] == 10000
    with pytest.raises(ValueError):
        cell_bounds(3, 4)
