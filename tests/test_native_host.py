"""libpert_hip.so without a GPU: it loads, exports every symbol include/pert_hip.h
declares, validates arguments before launching, and its per-(bin, cell) arithmetic
(pert_math.h, compiled for the host by the same hipcc build) matches the fp64 oracle.
"""
import os
import re

import numpy as np
import pytest
import torch
from scipy import special as sp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "pert_hip.h")


@pytest.fixture(scope="module")
def nat():
    from scdna_replication_tools_amd import build, _native
    build.build()
    _native.lib()
    return _native


def header_functions():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(pert_\w+)\s*\(", text, flags=re.M)))


def test_exports_every_header_symbol(nat):
    fns = header_functions()
    assert len(fns) >= 9
    lib = nat.lib()
    for f in fns:
        assert hasattr(lib, f), f
    assert set(fns) == set(nat.EXPORTED_SYMBOLS)
    assert b"gfx950" in lib.pert_version()


def test_struct_layout_matches_header(nat):
    import ctypes
    # pointers are 8-byte aligned after the int32 header fields
    assert ctypes.sizeof(nat.PertLayout) == 10 * 4
    assert nat.PertProblem.reads.offset == 9 * 4 + 4     # 9 int32 + padding to 8
    assert nat.PertState.params.offset == 40
    # 15 pointers, LT and variant, then the device-loop block
    assert nat.PertState.loop_ctl.offset == 40 + 15 * 8 + 2 * 4
    assert ctypes.sizeof(nat.PertState) == nat.PertState.loop_ctl.offset + 3 * 8 + 2 * 8 + 2 * 4


def test_layout_and_workspace(nat):
    lay = nat.make_layout(100, 37, 5, 2)
    assert lay.off_rho == 0 and lay.off_a == 100 and lay.off_lam == 101
    assert lay.n_shared == 100 + 2 + 2 * 2 * 5
    assert lay.off_tau + 37 == lay.n_params
    ncp, nbp, nblk, ncb = nat.workspace_sizes(2, 100, 37, 5, 2, 32)
    # 4 bin tiles + 1 level-1 row of pert_enum_step (groups of 8 >= sqrt(4) bin tiles)
    n_bt, n_g1, n_ct = 4, 1, 256 // 64
    assert ncp == (n_bt + n_g1) * (5 + 1) * 37 and nbp == n_ct * 100 and nblk == (n_bt + n_g1) * n_ct * 4
    # finalize's cell-block slots and arrival counter, then pert_enum_step's uint32 counters
    n_ctr = n_ct * n_g1 + n_ct + n_bt + 1
    assert ncb == ((37 + 63) // 64) * (2 * 2 * 5 + 2) + 1 + (n_ctr + 1) // 2
    # a genome-scale grid: 171 bin tiles in 13 groups of (at most) 14
    ncp2 = nat.workspace_sizes(2, 5451, 37, 5, 2, 32)[0]
    assert ncp2 == (171 + 13) * 6 * 37
    with pytest.raises(ValueError):
        nat.make_layout(0, 1, 5, 1)


def test_argument_validation_without_launch(nat):
    import ctypes
    pr = nat.PertProblem(kind=2, L=10, N=10, P=17, K1=5, n_libs=1, ldn=256)
    st = nat.PertState()
    hp = nat.PertAdamHparams()
    rc = nat.lib().pert_enum_pass(ctypes.byref(pr), ctypes.byref(st), ctypes.byref(hp), 0, None)
    assert rc != 0                      # P = 17 unsupported, null buffers: refused before any launch
    pr.P = 13
    rc = nat.lib().pert_enum_pass(ctypes.byref(pr), ctypes.byref(st), ctypes.byref(hp), 0, None)
    assert rc == 1                      # PERT_E_ARG (null pointers)


def test_host_comm_refuses_bad_arguments_and_times_out_alone(nat):
    """pert_comm_init_host: argument checks, and a rank whose peers never attach returns
    PERT_E_COMM_TIMEOUT after its deadline and leaves no segment in /dev/shm (no GPU needed:
    the attach comes before any HIP call)."""
    import ctypes
    import os
    import time
    lib = nat.lib_nogil()
    h = ctypes.c_void_p()
    name = "/pert-test-{}".format(os.getpid()).encode()
    assert lib.pert_comm_init_host(None, 2, 0, 16, 1.0, ctypes.byref(h)) == 1
    assert lib.pert_comm_init_host(b"no-slash", 2, 0, 16, 1.0, ctypes.byref(h)) == 1
    assert lib.pert_comm_init_host(name, 0, 0, 16, 1.0, ctypes.byref(h)) == 1
    assert lib.pert_comm_init_host(name, 2, 2, 16, 1.0, ctypes.byref(h)) == 1
    assert lib.pert_comm_init_host(name, 2, 0, 0, 1.0, ctypes.byref(h)) == 1
    assert lib.pert_comm_init_host(name, 2, 0, 16, 0.0, ctypes.byref(h)) == 1
    t0 = time.perf_counter()
    assert lib.pert_comm_init_host(name, 2, 0, 16, 0.3, ctypes.byref(h)) == nat.E_COMM_TIMEOUT
    assert 0.25 < time.perf_counter() - t0 < 5.0
    assert not h.value
    assert not os.path.exists("/dev/shm" + name.decode())
    assert lib.pert_comm_status(None) == 1 and lib.pert_comm_abort(None, 6) == 1
    assert lib.pert_comm_set_watchdog(None, None, 1.0) == 1 and lib.pert_comm_inject_fault(None, 0) == 1
    assert lib.pert_comm_wait_event(None, None, 0) == 1


def test_comm_loads_rccl_and_refuses_bad_arguments(nat):
    """pert_comm_load finds the RCCL this process already uses (torch's) and resolves its
    symbols; a unique id is made without a GPU; the sharded loop entry points refuse a null
    communicator and a grad_local aliasing grad_shared before any launch."""
    import ctypes
    from scdna_replication_tools_amd.engine import rccl_path
    lib = nat.lib_nogil()
    assert lib.pert_comm_load(b"/nonexistent/librccl.so") in (0, 5)   # 0 once an earlier call loaded it
    assert lib.pert_comm_load(rccl_path().encode()) == 0
    uid = (ctypes.c_uint8 * 128)()
    assert lib.pert_comm_unique_id(uid, 128) == 0 and any(bytes(uid))
    assert lib.pert_comm_unique_id(uid, 64) == 1
    assert lib.pert_comm_allreduce_sum_f64(None, None, None, 1, None) == 1
    assert lib.pert_comm_destroy(None) == 0
    pr = nat.PertProblem(kind=2, L=10, N=10, P=13, K1=5, n_libs=1, ldn=256)
    st = nat.PertState()
    hp = nat.PertAdamHparams()
    f = (ctypes.c_float * 4)()
    n = ctypes.c_int32()
    host = (ctypes.c_double * 8)()
    assert lib.pert_svi_steps_sharded(ctypes.byref(pr), ctypes.byref(st), ctypes.byref(hp), f, f, 0, 1, 0, None,
                                      None, None, None) == 1
    assert lib.pert_svi_run_sharded(ctypes.byref(pr), ctypes.byref(st), ctypes.byref(hp), f, f, 1, 8, 8, 0, None,
                                    None, None, host, ctypes.byref(n), None) == 1


def test_nb_lgdiff_host_matches_scipy(nat):
    rng = np.random.default_rng(1)
    d = np.concatenate([rng.uniform(1, 8, 2000), np.exp(rng.uniform(np.log(8), np.log(3e4), 4000))]).astype(np.float32)
    x = np.floor(np.exp(rng.uniform(0, np.log(2e4), d.size))).astype(np.float32)
    x[::5] = 0
    lam, psi = nat.selftest_nb_lgdiff_host(d, x)
    D, X = d.astype(np.float64), x.astype(np.float64)
    xlx = np.where(X > 0, X * np.log(np.where(X > 0, X, 1)), 0)
    lref = sp.gammaln(D + X) - sp.gammaln(D) - (xlx - X)
    pref = sp.digamma(D + X) - sp.digamma(D)
    assert (np.abs(lam - lref) / np.maximum(1.0, np.abs(lref))).max() < 2e-6
    assert (np.abs(psi - pref) / np.maximum(1e-3, np.abs(pref))).max() < 2e-5


@pytest.mark.parametrize("P", [13, 5])
def test_enum_cellbin_host_matches_autograd(nat, P):
    from torch.distributions import Bernoulli, Categorical, NegativeBinomial
    rng = np.random.default_rng(P)
    n = 300
    x = rng.integers(0, 400, n).astype(np.float32)
    st = rng.integers(0, P, n)
    em1 = np.zeros((n, P), np.float32)
    em1[np.arange(n), st] = 1e6 - 1
    S1 = em1.sum(1)
    z = (rng.normal(size=(n, P)) * 2).astype(np.float32)
    z[np.arange(n), st] += 5
    D = rng.uniform(0.3, 60, n).astype(np.float32)
    phi = rng.uniform(0.0002, 0.9998, n).astype(np.float32)
    lam = 0.75
    out = nat.selftest_enum_cellbin_host(P, x, em1, S1, z, np.log1p(-lam), D, phi)

    zt = torch.tensor(z, dtype=torch.float64, requires_grad=True)
    Dt = torch.tensor(D, dtype=torch.float64, requires_grad=True)
    pt = torch.tensor(phi, dtype=torch.float64, requires_grad=True)
    X = torch.tensor(x, dtype=torch.float64)
    pi = torch.softmax(zt, -1)
    phic = torch.where(pt < 0.001, torch.full_like(pt, 0.001), pt)
    phic = torch.where(phic > 0.999, torch.full_like(phic, 0.999), phic)
    cn = torch.arange(P).reshape(P, 1)
    rep = torch.tensor([0., 1.], dtype=torch.float64).reshape(2, 1, 1)
    delta = cn * (1 + rep) * Dt
    delta = torch.where(delta < 1, torch.ones_like(delta), delta)
    lp = (Categorical(pi).log_prob(cn) + Bernoulli(phic).log_prob(rep)
          + NegativeBinomial(delta, probs=torch.tensor(lam, dtype=torch.float64)).log_prob(X))
    E = torch.logsumexp(lp.reshape(2 * P, n), 0)
    xlx = torch.where(X > 0, X * torch.log(torch.where(X > 0, X, torch.ones_like(X))), torch.zeros_like(X))
    kappa = X * np.log(lam) + xlx - X - torch.lgamma(1 + X)
    dirv = (torch.tensor(em1, dtype=torch.float64) * torch.log(pi)).sum(-1)
    (E - kappa + dirv).sum().backward()

    assert np.abs(out["E"] - (E - kappa).detach().numpy()).max() < 2e-4
    # the Dirichlet variable part as the reference's fp32 value (pi32 = fl(exp / sum), its log):
    # within the fp32 quantisation of pi (W 2^-24 per element) of the fp64 value, and within a
    # few ulp of torch's fp32 evaluation (tests/test_dirichlet_value.py)
    # (an ulp of pi_jmax is W 2^-24 ~ 0.06 of the value; the fp32 row sum is off by a few ulp)
    q = np.float64(1e6 - 1) * 2.0 ** -24
    assert np.allclose(out["dirv"], dirv.detach().numpy(), rtol=1e-6, atol=8 * q)
    d32 = torch.xlogy(torch.tensor(em1), torch.softmax(torch.tensor(z), -1)).sum(-1).numpy()
    assert (np.abs(out["dirv"] - d32) <= 8 * q).mean() > 0.99
    rel = lambda a, b: np.linalg.norm(a - b) / np.linalg.norm(b)
    assert rel(out["gz"], zt.grad.numpy()) < 1e-6
    assert rel(out["gD"], Dt.grad.numpy()) < 1e-5
    assert rel(out["gt"], pt.grad.numpy() * phi * (1 - phi)) < 1e-5
    idx = torch.argmax(lp.reshape(2 * P, n), 0).numpy()
    assert (out["argmax"] == idx).mean() > 0.99


def test_argmax_logit_gradient_at_saturation(nat):
    """Once the prior has pushed a state so far that fp32 pi_argmax rounds to 1, the
    reference's fp32 autograd (SoftmaxTransform + Dirichlet + Categorical, the oracle's
    tensor algebra) still delivers the prior's pull W (1 - pi_argmax) on the argmax logit --
    through the gradient of the max subtraction, minus the other logits' sum -- and so do the
    kernels (pert_math.h jmax_grad).  The per-element form pi_k (S1 + sgm) - W_k - gcm_k rounds
    that pull to 0 here (tools/stop_probe.py: why the product's genome-length step 2 stopped 27
    iterations late)."""
    from torch.distributions import (Bernoulli, Categorical, Dirichlet, NegativeBinomial, constraints,
                                      transform_to)
    P, n = 13, 400
    rng = np.random.default_rng(7)
    x = rng.integers(50, 300, n).astype(np.float32)
    st = rng.integers(0, P, n)
    W = np.float32(1e6 - 1)
    em1 = np.zeros((n, P), np.float32)
    em1[np.arange(n), st] = W
    S1 = em1.sum(1)
    z = (rng.normal(size=(n, P)) * 0.5).astype(np.float32)
    z[np.arange(n), st] += rng.uniform(17.5, 21.0, n).astype(np.float32)      # fp32 pi_argmax ~ 1
    D = rng.uniform(20, 60, n).astype(np.float32)
    phi = rng.uniform(0.01, 0.99, n).astype(np.float32)
    lam = 0.75
    out = nat.selftest_enum_cellbin_host(P, x, em1, S1, z, np.log1p(-lam), D, phi)

    # the reference's arithmetic: fp32 torch autograd of the model's terms (oracle/pert_oracle.py)
    zt = torch.tensor(z, requires_grad=True)
    pi = transform_to(constraints.simplex)(zt)
    X = torch.tensor(x)
    cn = torch.arange(P).reshape(P, 1)
    rep = torch.tensor([0., 1.]).reshape(2, 1, 1)
    delta = torch.clamp(cn * (1 + rep) * torch.tensor(D), min=1.0)
    lp = (Categorical(pi).log_prob(cn) + Bernoulli(torch.tensor(phi)).log_prob(rep)
          + NegativeBinomial(delta, probs=torch.tensor(lam)).log_prob(X))
    E = torch.logsumexp(lp.reshape(2 * P, n), 0)
    (E.sum() + Dirichlet(torch.tensor(em1) + 1.0).log_prob(pi).sum()).backward()
    i = np.arange(n)
    ref = zt.grad.numpy()[i, st]
    pull = (np.float64(W) * (1.0 - torch.softmax(torch.tensor(z, dtype=torch.float64), -1).numpy()))[i, st]
    assert (pi.detach().numpy()[i, st] == 1.0).mean() > 0.6          # saturated in fp32
    assert np.median(pull) > 1e-2                                    # and the pull is not small
    got = out["gz"][i, st]
    assert np.abs(got - ref).max() < 2e-4, np.abs(got - ref).max()
    # the per-element form's value on these elements misses the pull
    old = (em1 - torch.softmax(torch.tensor(z), -1).numpy() * S1[:, None])[i, st]
    assert np.abs(old - ref).max() > 50 * 2e-4


def test_online_argmax_gradient_is_minus_the_others_sum(nat):
    """The three-wave pass's arithmetic (enum_online + enum_jmax, run on the host): the argmax
    logit's gradient is minus the sum of the other logits' gradients (a softmax gradient sums
    to zero), as in enum_forward -- 1 - pi_jmax is the others' pi summed with the same scaled
    exponentials and the same 1 / total, with no further correction -- and E equals
    enum_forward's.  Saturated rows (fp32 pi_argmax rounds to 1) included."""
    P, n = 13, 20000
    rng = np.random.default_rng(7)
    x = rng.integers(50, 300, n).astype(np.float32)
    st = rng.integers(0, P, n)
    em1 = np.zeros((n, P), np.float32)
    em1[np.arange(n), st] = np.float32(1e6 - 1)
    S1 = em1.sum(1)
    z = (rng.normal(size=(n, P)) * 0.5).astype(np.float32)
    z[np.arange(n), st] += rng.uniform(0.0, 63.0, n).astype(np.float32)
    D = rng.uniform(20, 60, n).astype(np.float32)
    phi = rng.uniform(0.01, 0.99, n).astype(np.float32)
    fwd = nat.selftest_enum_cellbin_host(P, x, em1, S1, z, np.log1p(-0.75), D, phi)
    onl = nat.selftest_enum_online_host(P, x, em1, S1, z, np.log1p(-0.75), D, phi)
    np.testing.assert_allclose(onl["E"], fwd["E"], rtol=0, atol=2e-6 * float(np.abs(fwd["E"]).max()))
    i = np.arange(n)
    eps = float(np.finfo(np.float32).eps)
    for out in (onl, fwd):
        g = out["gz"].astype(np.float64)
        gj = g[i, st]
        others = g.sum(1) - gj
        mag = np.abs(g).sum(1) - np.abs(gj)                 # the others' terms, before cancellation
        ulps = np.abs(gj + others) / (np.abs(others) * eps + 1e-30)
        ulps_mag = np.abs(gj + others) / (mag * eps + 1e-30)
        # the residual is the rounding of the others' pi summed two ways (a few ulps); a scale
        # correction on 1 - pi_jmax alone showed up here as up to ~1,300 ulps (p99 ~22)
        assert np.percentile(ulps, 99) < 4.0, np.percentile(ulps, 99)
        assert ulps_mag.max() < 64.0, ulps_mag.max()


@pytest.mark.parametrize("dlo,dhi", [(0.3, 1.3), (1.0, 1.6), (1.0, 5.0), (2.0, 7.0), (0.5, 12.0)])
def test_online_low_coverage_matches_cellbin(nat, dlo, dhi):
    """The low-coverage regime of the three-wave pass (D = u omega (1-lam)/lam below the
    asymptotic threshold, as 20 kb bins put it: chains chi D < 1 clamped, 1 <= chi D < 5 shifted
    -- two at a time in packed fp32 where both are -- and the rest asymptotic with the hoisted
    invariants) against enum_cellbin's per-chain nb_lgdiff: the same E and pi-logit gradient
    within fp32 rounding.  Counts 0..12 (zeros included), weak and strong prior rows."""
    P, n = 13, 20000
    rng = np.random.default_rng(11)
    x = rng.integers(0, 13, n).astype(np.float32)
    em1 = np.where(rng.random((n, P)) < 0.5, 0.0, rng.uniform(0, 5, (n, P))).astype(np.float32)
    st = rng.integers(0, P, n)
    strong = rng.random(n) < 0.5
    em1[np.arange(n)[strong], st[strong]] = np.float32(1e6 - 1)
    S1 = em1.sum(1)
    z = rng.normal(size=(n, P)).astype(np.float32)
    D = rng.uniform(dlo, dhi, n).astype(np.float32)
    phi = rng.uniform(0.01, 0.99, n).astype(np.float32)
    fwd = nat.selftest_enum_cellbin_host(P, x, em1, S1, z, np.log1p(-0.75), D, phi)
    onl = nat.selftest_enum_online_host(P, x, em1, S1, z, np.log1p(-0.75), D, phi)
    scale = np.maximum(1.0, np.abs(fwd["E"]))
    assert (np.abs(onl["E"] - fwd["E"]) / scale).max() < 1e-5
    g_scale = np.maximum(1.0, np.abs(fwd["gz"]).max(1, keepdims=True))
    assert (np.abs(onl["gz"] - fwd["gz"]) / g_scale).max() < 1e-5


def _host_comm_rank(rank, name, q):
    import ctypes
    import time
    from scdna_replication_tools_amd import _native
    lib = _native.lib_nogil()
    h = ctypes.c_void_p()
    rc = lib.pert_comm_init_host(name, 2, rank, 16, 10.0, ctypes.byref(h))
    out = {"init": rc}
    if rc == 0:
        if rank == 1:
            time.sleep(0.2)
            out["abort"] = lib.pert_comm_abort(h, _native.E_COMM_FAULT)
            out["status"] = lib.pert_comm_status(h)
        else:
            t0 = time.time()
            st = 0
            while st == 0 and time.time() - t0 < 10.0:
                st = lib.pert_comm_status(h)
                time.sleep(0.01)
            out["status"], out["waited"] = st, time.time() - t0
        out["destroy"] = lib.pert_comm_destroy(h)
    q.put((rank, out))


def test_host_comm_two_processes_share_the_abort_word(nat):
    """Two processes attach one host-staged communicator (no GPU needed before the first
    all-reduce): the segment is unlinked once both have mapped it, and an abort raised by rank 1
    is seen by rank 0 as PERT_E_COMM_ABORTED -- the word a failed rank's peers poll."""
    import multiprocessing as mp
    import os
    name = "/pert-test2-{}".format(os.getpid()).encode()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_host_comm_rank, args=(r, name, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=60) for _ in range(2))
    for p in ps:
        p.join(timeout=30)
    assert got[0]["init"] == 0 and got[1]["init"] == 0, got
    assert not os.path.exists("/dev/shm" + name.decode())
    assert got[1]["abort"] == 0 and got[1]["status"] == nat.E_COMM_FAULT
    assert got[0]["status"] == nat.E_COMM_ABORTED and got[0]["waited"] < 10.0
    assert got[0]["destroy"] == 0 and got[1]["destroy"] == 0
