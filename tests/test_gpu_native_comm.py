"""GPU: the library's own RCCL communicator (pert_comm, include/pert_hip.h) driving a sharded
fit's whole SVI loop in C (pert_svi_run_sharded / pert_svi_steps_sharded: reductions into the
shard's grad_local, the all-reduce queued on the fit's stream, Adam) against the same sharded
step driven per iteration from Python (PertShard with a Python all-reduce; the unsplit
pert_finalize + pert_adam sequence).  One GPU, so the
communicator is a one-rank RCCL world (a sum over one rank is the identity): both loops run
the same kernels on the same state, and the loss traces, the stopping iteration and the final
parameters must be identical bit for bit.  The multi-GPU bench runs the same path at N = 2..8.
"""
import time

import numpy as np
import pytest
import torch

from tests._problems import KIND_OF, init_constrained, make_problem

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def comm():
    from scdna_replication_tools_amd.engine import RcclComm
    c = RcclComm.world1()
    yield c
    c.close()


def _shard(kind, kw, z, **extra):
    from scdna_replication_tools_amd.engine import PertShard
    sh = PertShard(KIND_OF[kind], init=init_constrained(kind, z), device="cuda", **kw, **extra)
    sh.set_unconstrained({k: v.numpy() for k, v in z.items()})
    return sh


def _state(sh):
    out = {k: np.asarray(v) for k, v in sh.constrained().items()}
    if sh.z_pi is not None:
        out["z_pi"] = sh.z_pi.cpu().numpy()
    return out


def test_comm_allreduce_world1_is_identity(comm):
    t = torch.arange(5452, dtype=torch.float64, device="cuda") * 0.37
    want = t.clone()
    comm.allreduce(t)
    torch.cuda.synchronize()
    assert torch.equal(t, want)
    n = 200
    t0 = time.perf_counter()
    for _ in range(n):
        comm.allreduce(t)
    torch.cuda.synchronize()
    print("pert_comm all-reduce of 5,452 fp64 (world 1): {:.1f} us per call".format(
        (time.perf_counter() - t0) / n * 1e6))


# overlap: the split step (pert_finalize_shared, the all-reduce on the comm's side stream beside
# pert_finalize_cells_adam, pert_adam_shared) against the Python loop's pert_finalize + pert_adam;
# delay: with a 20 us stand-in kernel in every all-reduce
@pytest.mark.parametrize("kind,fused", [("step2", False), ("step2", True), ("step3", True), ("step1p", False),
                                        ("step3", False)])
@pytest.mark.parametrize("events,overlap,delay", [(False, True, 0.0), (True, True, 0.0), (False, False, 0.0),
                                                  (True, False, 20.0), (False, True, 20.0)])
def test_native_sharded_loop_matches_python_sharded_loop(comm, kind, fused, events, overlap, delay):
    comm.set_options(overlap=overlap, delay_us=delay)
    prob, kw, z = make_problem(kind, seed=4)
    a = _shard(kind, kw, z, fused=fused, comm=comm)
    b = _shard(kind, kw, z, fused=fused, allreduce=lambda t: None)     # per-iteration Python loop
    assert a.comm is comm and b.comm is None
    if events:
        a.pass_events, a.pass_event_stride = [], 3
    la, ra = a.run_svi(60, 12, 5e-2)
    lb, rb = b.run_svi(60, 12, 5e-2)
    assert (ra, len(la)) == (rb, len(lb))
    assert np.array_equal(np.asarray(la), np.asarray(lb))
    sa, sb = _state(a), _state(b)
    for k in sa:
        assert np.array_equal(sa[k], sb[k]), k
    if events:
        assert len(a.pass_events) >= len(la) // 3
    comm.set_options()


def test_rccl_comm_fault_aborts_and_a_new_comm_works():
    """The RCCL backend's failure path at world 1 (the only RCCL world a one-GPU box has): an
    all-reduce that cannot be queued (pert_comm_inject_fault) makes the C loop abort the
    communicator (ncclCommAbort) and raise CommError instead of hanging; the aborted comm
    refuses further work, closes cleanly, and a new communicator fits normally."""
    from scdna_replication_tools_amd import _native as nat
    from scdna_replication_tools_amd.engine import RcclComm
    prob, kw, z = make_problem("step2", seed=4)
    c = RcclComm.world1()
    a = _shard("step2", kw, z, comm=c)
    c.inject_fault(13)                               # iteration 12 (call 0: the shard's set-up all-reduce)
    with pytest.raises(nat.CommError) as e:
        a.run_svi(40, 10 ** 9, 0.0)
    assert e.value.code == nat.E_COMM_FAULT
    assert c.status() == nat.E_COMM_FAULT
    assert a.last_launched == 8                      # the first chunk was queued whole, the second not
    with pytest.raises(nat.CommError):
        a.run_svi(8, 10 ** 9, 0.0)                   # the aborted comm refuses further work
    c.close()
    c2 = RcclComm.world1()
    b = _shard("step2", kw, z, comm=c2)
    ref = _shard("step2", kw, z, allreduce=lambda t: None)
    lb, _ = b.run_svi(20, 10 ** 9, 0.0)
    lr, _ = ref.run_svi(20, 10 ** 9, 0.0)
    assert np.array_equal(np.asarray(lb), np.asarray(lr))
    c2.close()


def test_rccl_comm_raised_abort_word_stops_the_loop():
    """A raised abort word (what a failed peer on the node does) makes the loop return
    PERT_E_COMM_ABORTED at its first wait."""
    from scdna_replication_tools_amd import _native as nat
    from scdna_replication_tools_amd.engine import RcclComm
    prob, kw, z = make_problem("step2", seed=4)
    c = RcclComm.world1()
    a = _shard("step2", kw, z, comm=c)
    c.abort(nat.E_COMM_ABORTED)
    t0 = time.perf_counter()
    with pytest.raises(nat.CommError) as e:
        a.run_svi(40, 10 ** 9, 0.0)
    assert e.value.code == nat.E_COMM_ABORTED
    assert time.perf_counter() - t0 < 10.0
    c.close()
