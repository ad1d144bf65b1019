"""GPU: the one-launch SVI step of the three-wave pass (pert_enum_step, include/pert_hip.h)
against the same pass followed by the separate pert_finalize + pert_adam launches.

Both compute the same update; only the order of the fp32 partial sums differs (the fused
reductions sum bin tiles in groups of ~sqrt(n_bt), finalize in 16 interleaved groups), so
trajectories agree to rounding.  Cases cover a partial last cell tile, several libraries,
tile lengths that do not divide L, a group count with a partial last group, step 3 (rho and
a frozen) and the counters' re-arming over many launches.
"""
import numpy as np
import pytest
import torch

from tests._problems import KIND_OF, init_constrained, make_problem

pytestmark = pytest.mark.gpu


def _pair(kind, kw, z, **extra):
    from scdna_replication_tools_amd.engine import PertShard
    out = []
    for fused in (True, False):
        sh = PertShard(KIND_OF[kind], init=init_constrained(kind, z), device="cuda", variant=3, fused=fused,
                       **kw, **extra)
        sh.set_unconstrained({k: v.numpy() for k, v in z.items()})
        out.append(sh)
    return out


def _state(sh):
    out = {k: np.asarray(v, np.float64) for k, v in sh.constrained().items()}
    out["z_pi"] = sh.z_pi.cpu().numpy().astype(np.float64)
    return out


@pytest.mark.parametrize("kind,N,L,n_libs,lt", [
    ("step2", 40, 300, 2, 0),        # one partial cell tile, auto tile length
    ("step2", 130, 517, 3, 7),       # 3 cell tiles (last partial), 74 bin tiles: 9 groups of 9
    ("step3", 70, 257, 2, 11),       # rho, a frozen
    ("step2", 64, 64, 1, 64),        # one workgroup: every finalizer in the same wave
])
def test_fused_step_matches_separate_launches(kind, N, L, n_libs, lt):
    prob, kw, z = make_problem(kind, L=L, N=N, n_libs=n_libs, seed=31)
    a, b = _pair(kind, kw, z, bins_per_tile=lt)
    assert a.fused and not b.fused
    la = [a.step() for _ in range(12)]
    lb = [b.step() for _ in range(12)]
    np.testing.assert_allclose(la, lb, rtol=2e-6)
    sa, sb = _state(a), _state(b)
    for k in sa:
        np.testing.assert_allclose(sa[k], sb[k], rtol=2e-4, atol=2e-5, err_msg=k)


def test_fused_device_loop_stops_where_separate_launches_stop():
    prob, kw, z = make_problem("step2", seed=5)
    a, b = _pair("step2", kw, z)
    la, ra = a.run_svi(80, 15, 2e-2)
    lb, rb = b.run_svi(80, 15, 2e-2)
    assert ra == rb == 1 and len(la) == len(lb)
    np.testing.assert_allclose(la, lb, rtol=2e-6)
    ca, _ = a.decode()
    cb, _ = b.decode()
    assert (ca == cb).float().mean().item() >= 0.999
