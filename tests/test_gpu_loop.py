"""GPU: the device-side SVI loop (PertShard.run_svi, include/pert_hip.h loop_ctl) against
the host loop of reference pert_model.py:742-758 driven step by step.

Both loops run the same kernels on the same state, so the loss traces, the stopping
iteration and the final parameters must be identical bit for bit.
"""
import math

import numpy as np
import pytest
import torch

from tests._problems import KIND_OF, init_constrained, make_problem

pytestmark = pytest.mark.gpu


def _shard(kind, kw, z, **extra):
    from scdna_replication_tools_amd.engine import PertShard
    sh = PertShard(KIND_OF[kind], init=init_constrained(kind, z), device="cuda", **kw, **extra)
    sh.set_unconstrained({k: v.numpy() for k, v in z.items()})
    return sh


def _host_loop(sh, max_iter, min_iter, rel_tol):
    from scdna_replication_tools_amd.pert_model import _converged
    losses = []
    for i in range(max_iter):
        loss = sh.step()
        losses.append(loss)
        if _converged(losses, i, min_iter, rel_tol):
            return losses, 1
        if np.isnan(loss):
            return losses, 2
    return losses, 0


def _state(sh):
    out = {k: np.asarray(v) for k, v in sh.constrained().items()}
    if sh.z_pi is not None:
        out["z_pi"] = sh.z_pi.cpu().numpy()
    return out


# (variant, fused): the two-wave pass, the three-wave pass with separate finalize / adam
# launches (the default), and the three-wave pass as one launch per step (pert_enum_step)
VARIANTS = [(0, False), (3, False), (3, True)]


@pytest.mark.parametrize("variant,fused", VARIANTS)
@pytest.mark.parametrize("kind", ["step2", "step1", "step1p", "step3"])
@pytest.mark.parametrize("max_iter,min_iter,rel_tol", [(60, 12, 5e-2), (21, 5, 0.0)])
def test_device_loop_matches_host_loop(kind, max_iter, min_iter, rel_tol, variant, fused):
    if fused and kind.startswith("step1"):
        pytest.skip("step 1 has no one-launch form")
    prob, kw, z = make_problem(kind, seed=4)
    a = _shard(kind, kw, z, variant=variant, fused=fused)
    b = _shard(kind, kw, z, variant=variant, fused=fused)
    assert a.fused == fused
    la, ra = _host_loop(a, max_iter, min_iter, rel_tol)
    lb, rb = b.run_svi(max_iter, min_iter, rel_tol)
    assert ra == rb
    if rel_tol > 0:
        assert ra == 1 and len(la) < max_iter       # the plateau rule fired inside the budget
    assert lb == la                                 # identical fp64 loss records
    sa, sb = _state(a), _state(b)
    for k in sa:
        np.testing.assert_array_equal(sa[k], sb[k], err_msg=k)
    assert a.t == b.t
    # a further step continues the same Adam trajectory (step counters agree)
    assert a.step() == b.step()
    if not kind.startswith("step1"):
        ca, _ = a.decode()
        cb, _ = b.decode()
        assert torch.equal(ca, cb)


@pytest.mark.parametrize("variant,fused", VARIANTS)
def test_device_loop_stops_on_nan(variant, fused):
    prob, kw, z = make_problem("step2", seed=6)
    z = dict(z)
    u = z["expose_u"].clone()
    u[3] = float("nan")
    z["expose_u"] = u
    sh = _shard("step2", kw, z, variant=variant, fused=fused)
    losses, reason = sh.run_svi(30, 5, 1e-6)
    assert reason == 2 and len(losses) == 1 and math.isnan(losses[0])
    assert sh.t == 1


@pytest.mark.parametrize("variant,fused", VARIANTS)
@pytest.mark.parametrize("kind", ["step2", "step1p"])
def test_chunked_loop_equals_per_step_launches(kind, variant, fused):
    """run_svi's one-call chunks (pert_svi_steps through the GIL-releasing handle), with and
    without the per-pass timing events, equal the per-step launch sequence bit for bit."""
    if fused and kind.startswith("step1"):
        pytest.skip("step 1 has no one-launch form")
    prob, kw, z = make_problem(kind, seed=5)
    per_step = _shard(kind, kw, z, variant=variant, fused=fused)
    per_step._lib_chunk = None                      # the per-iteration launches of _launch_step
    la, ra = per_step.run_svi(19, 10 ** 9, 0.0)
    b = _shard(kind, kw, z, variant=variant, fused=fused)
    lb, rb = b.run_svi(19, 10 ** 9, 0.0)
    c = _shard(kind, kw, z, variant=variant, fused=fused)
    c.pass_events = []
    lc, rc = c.run_svi(19, 10 ** 9, 0.0)
    assert la == lb == lc and ra == rb == rc == 0
    assert len(c.pass_events) == 19 and all(e0.elapsed_time(e1) > 0 for e0, e1 in c.pass_events)
    sa, sb, sc = _state(per_step), _state(b), _state(c)
    for k in sa:
        np.testing.assert_array_equal(sa[k], sb[k], err_msg=k)
        np.testing.assert_array_equal(sa[k], sc[k], err_msg=k)


def test_device_loop_chunk_boundaries():
    """Stopping iterations on either side of a read-back chunk boundary."""
    prob, kw, z = make_problem("step2", seed=8)
    ref = _shard("step2", kw, z)
    full, _ = ref.run_svi(40, 10 ** 9, 0.0)
    for n in (7, 8, 9, 17):
        sh = _shard("step2", kw, z)
        losses, reason = sh.run_svi(n, 10 ** 9, 0.0, chunk=8, depth=1)
        assert reason == 0 and losses == full[:n]
