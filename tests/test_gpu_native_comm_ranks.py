"""GPU: the product's sharded C loop (pert_svi_run_sharded: reductions into grad_local, the
all-reduce queued by the library on the fit's stream, Adam) at world 2 -- two ranks sharing
GPU 0, joined by the library's host-staged communicator (pert_comm_init_host; RCCL refuses
two ranks on one GPU) -- against

* the same shards driven per iteration from Python over gloo (the two-rank sum commutes, so
  the trajectories must be identical bit for bit), and the single-rank fit (summation order);
* every rank stopping after the same chunk (equal iterations queued);
* a fault injected on rank 1's all-reduce k: rank 1 raises at once, rank 0 raises within 10 s
  through the node's abort word (not its 600 s deadline);
* a peer that never arrives: rank 0 raises at the communicator's deadline.

Reference: pert_model.py:800-816 (the svi_s.step() loop a shard runs); SURVEY.md section 8e.
"""
import os
import socket
import time

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

ITERS, MIN_ITER, REL_TOL, SEED = 40, 15, 2e-2, 17


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
    for k in ("cn_obs", "rep_obs"):
        if k in kw and kw[k] is not None:
            k2[k] = np.asarray(kw[k])[:, sl]
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


def _shard(kind, kw, z, **extra):
    from scdna_replication_tools_amd.engine import PertShard
    from tests._problems import KIND_OF, init_constrained
    sh = PertShard(KIND_OF[kind], init=init_constrained(kind, {k: torch.as_tensor(v) for k, v in z.items()}),
                   device="cuda:0", **kw, **extra)
    sh.set_unconstrained(z)
    return sh


def _state(sh):
    out = {k: np.asarray(v) for k, v in sh.constrained().items()}
    if sh.z_pi is not None:
        out["z_pi"] = sh.z_pi.cpu().numpy()
    return out


def _run_shards(kind, fused, rank, world, **extra):
    from scdna_replication_tools_amd.sharding import shard_slice
    from tests._problems import make_problem
    prob, kw, z = make_problem(kind, seed=SEED)
    N = np.asarray(kw["reads"]).shape[1]
    k2, z2 = _shard_inputs(kw, z, shard_slice(N, world, rank))
    return _shard(kind, k2, z2, is_root=(rank == 0), n_cells_total=N, fused=fused, **extra)


def _worker(rank, world, port, out_dir, mode, kind, fused):
    from scdna_replication_tools_amd import _native as nat
    from scdna_replication_tools_amd.engine import HostComm
    from scdna_replication_tools_amd.sharding import make_allreduce
    if mode == "deadline":
        os.environ["PERT_COMM_TIMEOUT_S"] = "3"
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:{}".format(port), rank=rank, world_size=world)
    out = {}
    try:
        torch.cuda.set_device(0)
        comm = HostComm()
        if mode == "match":
            a = _run_shards(kind, fused, rank, world, comm=comm)
            la, ra = a.run_svi(ITERS, MIN_ITER, REL_TOL)
            out.update(losses=la, reason=ra, launched=a.last_launched, native=_state(a))
            b = _run_shards(kind, fused, rank, world, allreduce=make_allreduce())     # Python loop, gloo
            lb, rb = b.run_svi(ITERS, MIN_ITER, REL_TOL)
            out.update(losses_py=lb, reason_py=rb, python=_state(b))
            if kind != "step1":
                cn, rep = a.decode()
                out.update(cn=cn.cpu().numpy(), rep=rep.cpu().numpy())
        else:
            a = _run_shards(kind, fused, rank, world, comm=comm)
            if mode == "fault" and rank == 1:
                comm.inject_fault(comm_calls_before_fault(a))
            if mode == "deadline" and rank == 1:
                time.sleep(12)                     # never reaches the fit's all-reduces
            else:
                t0 = time.time()
                try:
                    a.run_svi(400, 400, 0.0)
                    out["raised"] = None
                except nat.CommError as e:
                    out.update(raised=e.code, msg=str(e))
                out.update(t_start=t0, t_raise=time.time(), launched=a.last_launched)
        comm.close()
    finally:
        torch.save(_tensors(out), os.path.join(out_dir, "{}{}.pt".format(mode, rank)))
        dist.destroy_process_group()


def _tensors(v):
    if isinstance(v, dict):
        return {k: _tensors(x) for k, x in v.items()}
    return torch.as_tensor(v) if isinstance(v, np.ndarray) else v


def comm_calls_before_fault(shard):
    """Fail rank 1's all-reduce of SVI iteration 20: the set-up constants' calls come first."""
    return 20 + 1


def _spawn(mode, tmp_path, kind="step2", fused=False, limit=120):
    ctx = mp.spawn(_worker, args=(2, _free_port(), str(tmp_path), mode, kind, fused), nprocs=2, join=False)
    deadline = time.time() + limit
    while not ctx.join(timeout=2):
        if time.time() > deadline:
            for p in ctx.processes:
                if p.is_alive():
                    p.kill()
            pytest.fail("the two ranks did not finish within {} s".format(limit))
    r = [torch.load(str(tmp_path / "{}{}.pt".format(mode, i)), weights_only=True) for i in range(2)]
    return [_arrays(x) for x in r]


def _arrays(v):
    if isinstance(v, dict):
        return {k: _arrays(x) for k, x in v.items()}
    return v.numpy() if isinstance(v, torch.Tensor) else v


@pytest.mark.parametrize("kind,fused", [("step2", False), ("step2", True), ("step3", False), ("step1", False)])
def test_native_loop_two_ranks_matches_python_loop_and_one_rank(tmp_path, kind, fused):
    r = _spawn("match", tmp_path, kind, fused)
    for i in range(2):
        # the C loop with the library's all-reduce == the per-step Python loop over gloo, bit for bit
        assert r[i]["reason"] == r[i]["reason_py"]
        assert np.array_equal(np.asarray(r[i]["losses"]), np.asarray(r[i]["losses_py"]))
        for k in r[i]["native"]:
            assert np.array_equal(r[i]["native"][k], r[i]["python"][k]), (i, k)
    # one global trajectory, the same stopping iteration and the same chunks queued on both ranks
    assert r[0]["losses"] == r[1]["losses"]
    assert r[0]["reason"] == r[1]["reason"]
    assert r[0]["launched"] == r[1]["launched"] >= len(r[0]["losses"])
    assert r[0]["launched"] % 8 == 0 or r[0]["launched"] == ITERS
    # against the single-rank fit of the whole problem (summation order only)
    from tests._problems import make_problem
    prob, kw, z = make_problem(kind, seed=SEED)
    one = _shard(kind, *_shard_inputs(kw, z, slice(None)), fused=fused)
    l1, r1 = one.run_svi(ITERS, MIN_ITER, REL_TOL)
    assert r[0]["reason"] == r1 and len(r[0]["losses"]) == len(l1)
    np.testing.assert_allclose(r[0]["losses"], l1, rtol=1e-6)
    if kind != "step1":
        cn, rep = (a.cpu().numpy() for a in one.decode())
        cn2 = np.concatenate([r[i]["cn"] for i in range(2)], axis=1)
        rep2 = np.concatenate([r[i]["rep"] for i in range(2)], axis=1)
        assert ((cn2 == cn) & (rep2 == rep)).mean() >= 0.999


def test_fault_on_one_rank_stops_every_rank(tmp_path):
    from scdna_replication_tools_amd import _native as nat
    r = _spawn("fault", tmp_path)
    assert r[1]["raised"] == nat.E_COMM_FAULT, r[1]
    assert r[0]["raised"] == nat.E_COMM_ABORTED, r[0]
    assert r[0]["t_raise"] - r[1]["t_raise"] < 10.0, (r[0]["t_raise"], r[1]["t_raise"])
    print("rank 0 raised {:.3f} s after rank 1".format(r[0]["t_raise"] - r[1]["t_raise"]))


def test_missing_peer_raises_at_the_deadline(tmp_path):
    from scdna_replication_tools_amd import _native as nat
    r = _spawn("deadline", tmp_path)
    assert r[0]["raised"] in (nat.E_COMM_TIMEOUT, nat.E_COMM_ABORTED), r[0]
    took = r[0]["t_raise"] - r[0]["t_start"]
    assert took < 10.0, took
    print("rank 0 raised {:.3f} s into its fit (deadline 3 s, counted from the set-up all-reduce)".format(took))
