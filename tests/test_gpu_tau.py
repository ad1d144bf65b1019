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


def _norm(reads, states):
    x, st = torch.as_tensor(reads), torch.as_tensor(states)
    return x / torch.where(st > 0.0, st, (torch.ones(x.shape) * 0.5).type(torch.float32))


@pytest.mark.parametrize("L,n_s,n_g,seed,reads_per_bin", [(271, 150, 50, 1, None), (5451, 64, 32, 2, None),
                                                          (1000, 96, 32, 3, 8)])
def test_kernel_matches_tensor_program(L, n_s, n_g, seed, reads_per_bin):
    """Same labels, flags and GMM means (to fp64 rounding) as the tensor program, for both
    tie directions; the low-coverage case (8 reads per bin) is full of exact ties."""
    reads, states = _profiles(n_s, n_g, L, seed, None if reads_per_bin is None else reads_per_bin * L)
    norm = _norm(reads, states).cuda()
    got = tau_init.kmeans_em_native(norm)
    X, Xc = tau_init._standardize(norm)
    for r, tie in enumerate((tau_init.TIE, -tau_init.TIE)):
        mu, fr, pp, lab = tau_init._kmeans_em(X, Xc, tie)
        g_mu, g_fr, g_pp, g_lab = got[r]
        assert torch.equal(g_lab, lab), (r, int((g_lab != lab).any(0).sum()))
        assert torch.equal(g_pp, pp), r
        assert torch.equal(g_fr, fr), r
        torch.testing.assert_close(g_mu, mu, rtol=1e-9, atol=1e-12)


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
