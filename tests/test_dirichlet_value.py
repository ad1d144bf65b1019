"""The Dirichlet site's VALUE as the reference's fp32 arithmetic forms it (CPU tests).

torch.distributions.Dirichlet.log_prob evaluates, per (bin, cell) element,
    xlogy(eta - 1, pi).sum(-1) + lgamma(eta.sum(-1)) - lgamma(eta).sum(-1)
in fp32.  With a g1_clones / composite prior lgamma(sum eta) is ~1.3e7 (ulp 1), so every
element's value is rounded to an integer before the sum, and in the late iterations of a fit,
where the pi logits of thousands of elements move in lockstep, the loss drops in steps of ~3.5e5
(one unit per element).  The reference's stopping rule sees those steps
(tools/stop_probe.py: a loss record without them stops the genome-length step 2 at 1,178 /
1,187 instead of 1,151).  The kernels reproduce the rounding: each element adds
q = fl(xs + A) - A to the loss, A = fl(lgamma(sum eta)) of its eta row (the table's last
column), xs = sum_k (eta_k - 1) log pi32_k with pi32_jmax = fl(1 / s) and s the fp32 row sum
of exp(z - max) in torch's CPU order; the host adds C = A - B per element (the torch32
normaliser), and fl(fl(xs + A) - B) = q + C exactly.
"""
import numpy as np
import pytest
import torch

from scdna_replication_tools_amd import _native
from scdna_replication_tools_amd.engine import EtaCodebook


def _torch_order(P):
    split = 8 if 9 <= P <= 15 else (4 if P == 5 else 0)
    return list(range(split, P)) + list(range(split))


@pytest.mark.parametrize("P", [9, 13, 15])
def test_torch_row_sum_order(P):
    """torch's fp32 CPU sum over a contiguous last dim of P values (9 <= P <= 15) adds the
    elements in the order the kernels assume (pert_math.h torch_row_sum_index): 8 .. P-1,
    then 0 .. 7 (sequentially, one rounding per addition)."""
    torch.set_num_threads(1)
    rng = np.random.default_rng(P)
    n = 4000
    z = (rng.normal(size=(n, P)) * 0.5).astype(np.float32)
    z[np.arange(n), rng.integers(0, P, n)] += rng.uniform(13, 18, n).astype(np.float32)
    e = torch.tensor(z)
    e = (e - e.max(-1, keepdim=True)[0]).exp()
    ref = e.sum(-1).numpy()
    acc = np.zeros(n, np.float32)
    for k in _torch_order(P):
        acc = (acc + e.numpy()[:, k]).astype(np.float32)
    assert np.array_equal(acc, ref)


@pytest.fixture(scope="module")
def nat():
    try:
        _native.lib()
    except Exception as exc:                                   # pragma: no cover
        pytest.skip("libpert_hip.so not built: {}".format(exc))
    return _native


def test_dirichlet_xlogy_value_matches_torch_fp32(nat):
    """The kernels' xs (host build of pert_math.h) against torch's fp32
    xlogy(eta - 1, softmax(z)).sum(-1) for g1_clones rows, saturated and not."""
    P, n = 13, 3000
    rng = np.random.default_rng(3)
    st = rng.integers(0, P, n)
    W = np.float32(1e6 - 1)
    em1 = np.zeros((n, P), np.float32)
    em1[np.arange(n), st] = W
    z = (rng.normal(size=(n, P)) * 0.5).astype(np.float32)
    z[np.arange(n), st] += rng.uniform(2.0, 20.0, n).astype(np.float32)
    out = nat.selftest_enum_cellbin_host(P, rng.integers(50, 300, n).astype(np.float32), em1, em1.sum(1), z,
                                         np.log1p(-0.75), rng.uniform(20, 60, n).astype(np.float32),
                                         rng.uniform(0.01, 0.99, n).astype(np.float32))
    pi = torch.distributions.transform_to(torch.distributions.constraints.simplex)(torch.tensor(z))
    ref = torch.xlogy(torch.tensor(em1), pi).sum(-1).numpy()
    got = out["dirv"]
    ulp = np.spacing(np.abs(ref).astype(np.float32))
    err = np.abs(got - ref) / ulp
    # where the rounding of pi_jmax matters: pi32_jmax itself is torch's (the value moves in
    # steps of W 2^-24 ~ 0.06 there), its log within 2 ulp (torch's vectorised logf and the
    # kernels' series differ in the last bit at ties; 1e-8 against the site's grid of 1)
    om = 1.0 - pi.numpy()[np.arange(n), st]
    sat = om < 1e-4                                          # s - 1 < 2^-13: fl(1 / s) = 2 - s
    assert sat.sum() > 500 and (err[sat] <= 2).mean() > 0.999, err[sat].max()
    # above, -log(s): off by the quotient's rounding, at most W 2^-24 (no lockstep there)
    # everywhere: the quotient's rounding (W 2^-24) and a few ulp of other libms' exp / log
    assert (np.abs(got - ref) <= float(W) * 2.0 ** -24 + 8 * ulp).mean() > 0.999
    # and the rounded site value: fl(fl(xs + A) - B) = (fl(xs + A) - A) + (A - B)
    eta = torch.tensor(em1 + 1.0)
    A = torch.lgamma(eta.sum(-1)).numpy()
    B = torch.lgamma(eta).sum(-1).numpy()
    site = (torch.tensor(ref) + torch.tensor(A) - torch.tensor(B)).numpy()   # torch's own order
    q = ((got + A).astype(np.float32) - A).astype(np.float32)
    same = q.astype(np.float64) + (A.astype(np.float64) - B) == site
    assert same[sat].mean() > 0.999 and same.mean() > 0.99, (same[sat].mean(), same.mean())


def test_kernel_table_rounding_column():
    """kernel_table(): eta - 1, S1, then A = fl32(lgamma(fl32(sum eta))) (torch's value) for the
    reference's rounding of the site value ('torch32'), 0 for the exact normaliser."""
    cb = EtaCodebook.from_states(np.array([[0, 3], [12, 5]]), 1e6, 13)
    t = cb.kernel_table()
    assert t.shape == (13, 15)
    A = torch.lgamma(torch.tensor(cb.table).sum(-1)).numpy()
    assert np.array_equal(t[:, 14], A)
    assert np.array_equal(t[:, 13], (cb.table.astype(np.float64) - 1).sum(1).astype(np.float32))
    assert np.all(cb.kernel_table(round_site=False)[:, 14] == 0)
