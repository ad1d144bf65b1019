"""GPU: the cell-sharded multi-rank fit (what bench.py / the fit run over RCCL on a node) with
two ranks sharing one GPU over gloo -- the same PertShard code path, all-reduce and device-side
SVI loop as N GPUs -- against the single-rank fit of the whole problem.

The ranks' loss is the all-reduced global loss, so both ranks record the same trajectory and
stop at the same iteration; it must match the single-rank run to fp summation-order noise, and
the decode must agree.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

KIND, SEED, ITERS, MIN_ITER, REL_TOL = "step2", 17, 40, 15, 2e-2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _shard_inputs(kw, z, sl):
    from scdna_replication_tools_amd.engine import EtaCodebook
    k2 = dict(kw)
    k2["reads"] = np.asarray(kw["reads"])[:, sl]
    k2["libs"] = np.asarray(kw["libs"])[sl]
    if "eta" in kw:
        k2["eta"] = EtaCodebook(np.ascontiguousarray(kw["eta"].codes[:, sl]), kw["eta"].table)
    z2 = {}
    for name, v in z.items():
        v = v.numpy()
        if name in ("expose_tau", "expose_u", "expose_betas"):
            v = v[sl]
        elif name == "expose_pi":
            v = v[:, sl]
        z2[name] = v
    return k2, z2


def _run(kw, z, **extra):
    from oracle import pert_oracle as po
    from scdna_replication_tools_amd.engine import PertShard
    from tests._problems import KIND_OF
    init = {k: v for k, v in po.constrain(KIND, {k: torch.as_tensor(v) for k, v in z.items()}).items()}
    init = {k: v.detach().numpy() for k, v in init.items()}
    sh = PertShard(KIND_OF[KIND], init=init, device="cuda:0", **kw, **extra)
    sh.set_unconstrained(z)
    losses, reason = sh.run_svi(ITERS, MIN_ITER, REL_TOL)
    # the all-reduce is idempotent: launches queued past the device-side stop leave the
    # reduced loss at the stopping iteration's value (not multiplied by the world size)
    assert sh.device_loss() == losses[-1], (sh.device_loss(), losses[-1])
    cn, rep = sh.decode()
    return losses, reason, cn.cpu().numpy(), rep.cpu().numpy(), sh.constrained()


def _worker(rank, world, port, out_dir, variant, fused):
    from scdna_replication_tools_amd.sharding import make_allreduce, shard_slice
    from tests._problems import make_problem
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:{}".format(port), rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        prob, kw, z = make_problem(KIND, seed=SEED)
        N = np.asarray(kw["reads"]).shape[1]
        sl = shard_slice(N, world, rank)
        k2, z2 = _shard_inputs(kw, z, sl)
        losses, reason, cn, rep, c = _run(k2, z2, is_root=(rank == 0), n_cells_total=N, allreduce=make_allreduce(),
                                          variant=variant, fused=fused)
        torch.save({"losses": losses, "reason": reason, "cn": torch.as_tensor(cn), "rep": torch.as_tensor(rep),
                    "rho": torch.as_tensor(c["expose_rho"]), "tau": torch.as_tensor(c["expose_tau"])},
                   os.path.join(out_dir, "r{}.pt".format(rank)))
    finally:
        dist.destroy_process_group()


# (variant, fused): the two-wave pass; the three-wave pass with separate launches (the
# default); the one-launch step, sharded: pert_enum_step(update_shared=0) -> all-reduce of
# the shared block -> pert_adam_shared
@pytest.mark.parametrize("variant,fused", [(0, False), (3, False), (3, True)])
def test_two_ranks_match_single_rank(tmp_path, variant, fused):
    from scdna_replication_tools_amd.sharding import shard_slice
    from tests._problems import make_problem
    mp.spawn(_worker, args=(2, _free_port(), str(tmp_path), variant, fused), nprocs=2, join=True)
    r = [torch.load(str(tmp_path / "r{}.pt".format(i)), weights_only=True) for i in range(2)]
    prob, kw, z = make_problem(KIND, seed=SEED)
    k1, z1 = _shard_inputs(kw, z, slice(None))
    losses, reason, cn, rep, c = _run(k1, z1, variant=variant, fused=fused)
    assert r[0]["losses"] == r[1]["losses"]                  # one global trajectory on every rank
    assert r[0]["reason"] == r[1]["reason"] == reason
    assert len(r[0]["losses"]) == len(losses)                # same stopping iteration
    np.testing.assert_allclose(r[0]["losses"], losses, rtol=1e-6)
    N = cn.shape[1]
    cn2 = np.concatenate([r[i]["cn"].numpy() for i in range(2)], axis=1)
    rep2 = np.concatenate([r[i]["rep"].numpy() for i in range(2)], axis=1)
    assert ((cn2 == cn) & (rep2 == rep)).mean() >= 0.999
    np.testing.assert_allclose(r[0]["rho"].numpy(), c["expose_rho"], rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(r[1]["rho"].numpy(), c["expose_rho"], rtol=1e-4, atol=1e-6)
    tau2 = np.concatenate([r[i]["tau"].numpy() for i in range(2)])
    np.testing.assert_allclose(tau2, c["expose_tau"], rtol=1e-4, atol=1e-6)
    assert shard_slice(N, 2, 1).stop == N

