"""GPU: the tau initialiser's k-means / EM stage as one HIP launch (pert_tau_kmeans_em,
csrc/tau_kernels.hip) against the tensor program it replaces (tau_init._kmeans_em, the same
algorithm as ~20 launches per iteration), and the product entry point on the GPU
(guess_times_batched on cuda: kernel + levels / scan + exact host path for the flagged
cells) against the per-cell sklearn restatement of the reference (prep.guess_times,
pert_model.py:364-457) for every cell."""
import time

import numpy as np
import pytest
import torch

from scdna_replication_tools_amd import prep, tau_init

pytestmark = pytest.mark.gpu


def _profiles(n_s, n_g, L, seed, num_reads=None):
    from scdna_replication_tools_amd.simulator import simulate
    sim = simulate(n_s=n_s, n_g=n_g, n_bins=L, num_reads=num_reads or 183 * L, seed=seed)
    reads = np.concatenate([sim.reads_s, sim.reads_g], axis=1).astype(np.float32)
    states = np.concatenate([sim.cn_s, sim.cn_g], axis=1).astype(np.float32)
    return reads, states


def _scale_mixture(L=600, N=60, seed=5):
    """Profiles whose 2-component GMM means come out closer than MEAN_GAP_THRESH, so the levels
    are percentiles chosen by the skew (pert_model.py:386-399): a symmetric scale mixture (mid),
    with an exponential right tail (early) or left tail (late); integer-valued like read counts.
    (reads, states) with states = 1, i.e. the profile is the CN-normalised reads."""
    rng = np.random.default_rng(seed)
    cols = []
    for n in range(N):
        x = rng.standard_normal(L) * np.where(rng.random(L) < 0.2, 4.0, 1.0)
        if n % 3 == 1:
            x = x + rng.exponential(3.0, L) * (rng.random(L) < 0.3)
        elif n % 3 == 2:
            x = x - rng.exponential(3.0, L) * (rng.random(L) < 0.3)
        cols.append(np.round(200 + 20 * x))
    reads = np.stack(cols, 1).astype(np.float32)
    return reads, np.ones_like(reads)


def _norm(reads, states):
    x, st = torch.as_tensor(reads), torch.as_tensor(states)
    return x / torch.where(st > 0.0, st, (torch.ones(x.shape) * 0.5).type(torch.float32))


@pytest.mark.parametrize("L,n_s,n_g,seed,reads_per_bin", [(271, 150, 50, 1, None), (5451, 64, 32, 2, None),
                                                          (1000, 96, 32, 3, 8), (600, 0, 0, 5, "mixture")])
def test_kernel_matches_tensor_program(L, n_s, n_g, seed, reads_per_bin):
    """The one-launch batched pass against the tensor programs it replaces (_kmeans_em, then
    _levels_scan), both tie directions: the same k-means labels and k-means++ / Lloyd / EM flags,
    the GMM means to fp64 rounding, and -- on every cell neither side flags (the flagged ones go
    to the exact host path) -- the same replicated fraction.  The low-coverage case (8 reads per
    bin) is full of exact ties; the G1/2-heavy case exercises the percentile levels (close GMM
    means) on most cells."""
    if reads_per_bin == "mixture":
        reads, states = _scale_mixture(L, 60, seed)
    else:
        reads, states = _profiles(n_s, n_g, L, seed, None if reads_per_bin is None else reads_per_bin * L)
    norm = _norm(reads, states).cuda()
    got = tau_init.binarize_native(norm)
    X, Xc = tau_init._standardize(norm)
    close = 0
    for r, tie in enumerate((tau_init.TIE, -tau_init.TIE)):
        mu, fr, pp, lab = tau_init._kmeans_em(X, Xc, tie)
        f, fr2, sc, mn = tau_init._levels_scan(X, Xc, mu, fr)
        g = got[r]
        assert torch.equal(g["labels"], lab), (r, int((g["labels"] != lab).any(0).sum()))
        assert torch.equal(g["pp"], pp), r
        torch.testing.assert_close(g["mu"], mu, rtol=1e-9, atol=1e-12)
        assert torch.equal(g["fragile"], fr2), r
        flagged = g["fragile"] | g["pp"] | g["scan"] | (g["minor"] > 0) | fr2 | pp | sc | (mn > 0)
        # as counts: torch divides by the scalar L as a multiplication by 1/L (1 ulp off the
        # reference's sum / len; the kernel divides)
        bad = (torch.round(g["frac"] * L) != torch.round(f * L)) & ~flagged
        assert not bool(bad.any()), (r, int(bad.sum()), ((g["frac"] - f)[bad] * L)[:8].tolist(),
                                     g["frac"][bad][:4].tolist(), f[bad][:4].tolist())
        # the scan margins agree except where a sum's last bits differ (fixed-point vs fp64)
        assert int((g["scan"] != sc).sum()) <= max(1, int(0.01 * norm.shape[1])), r
        close += int(((mu[0] - mu[1]).abs() < tau_init.MEAN_GAP_THRESH).sum())
    print("cells with percentile levels:", close // 2, "of", norm.shape[1])
    if reads_per_bin == "mixture":
        assert close // 2 >= 20


def test_guess_times_percentile_levels_match_reference_every_cell():
    """Cells whose levels are percentiles (close GMM means; early / mid / late by the skew):
    the product on the GPU equals the per-cell reference restatement for every cell."""
    reads, states = _scale_mixture(600, 60, 5)
    t_b = tau_init.guess_times_batched(reads, states, upsilon=6, device="cuda")[0]
    np.testing.assert_array_equal(t_b, prep.guess_times(reads, states, upsilon=6)[0])


@pytest.mark.parametrize("seed,L,n_s,n_g", [(6, 271, 300, 100), (11, 5451, 192, 64)])
def test_guess_times_on_gpu_matches_reference_every_cell(seed, L, n_s, n_g):
    reads, states = _profiles(n_s, n_g, L, seed)
    t_b, a_b, _ = tau_init.guess_times_batched(reads, states, upsilon=6, device="cuda")
    timings = dict(tau_init.guess_times_batched.last_timings)
    t_r, a_r, _ = prep.guess_times(reads, states, upsilon=6)
    np.testing.assert_array_equal(t_b, t_r)
    np.testing.assert_array_equal(a_b, a_r)
    print("guess_times on the GPU", L, "bins", reads.shape[1], "cells:", timings)


def test_guess_times_c1_size_is_fast():
    """configs[0]'s stand-in size (400 cells x 271 bins): the whole initialiser well under
    the 1.1 s the tensor program took there."""
    reads, states = _profiles(400, 0 + 1, 271, 0)
    tau_init.guess_times_batched(reads, states, 6, device="cuda")      # warm-up (module load, first launch)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tau_init.guess_times_batched(reads, states, 6, device="cuda")
    dt = time.perf_counter() - t0
    print("C1-size guess_times", dt, tau_init.guess_times_batched.last_timings)
    assert dt < 0.5
