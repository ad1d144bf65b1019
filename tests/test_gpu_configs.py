"""GPU parity at the shapes of BASELINE.json's configs,
every gradient element inside the Appendix C bound (tests/_bounds.py) against the fp64
oracle.

* configs[2] / configs[3] (C3 / C4): the full 5,451-bin 500 kb genome at the configs'
  coverage (1e6 reads per cell), a 64-cell shard, clone and composite priors -- including the
  reference's default g1_composite prior exactly as the product builds it (prep + code book,
  tests/_problems.py prior="product_composite") -- steps 1-3;
* configs[4] (C5): an 8-cell shard of the 136,275-bin 20 kb grid (about 7 reads per bin,
  the small-delta NB branch);
* C4 at full size (10,000 cells x 5,451 bins) through the product's pass: the per-cell
  gradients of cells sampled across the grid (first, middle, last partial wave tile)
  against the oracle on those cells, and the shared gradients against the sum over four
  disjoint shards (linearity of the cell plate);
* the C4 full-size step-2 fit against simulator truth.
"""
import numpy as np
import pytest
import torch

from oracle import pert_oracle as po
from tests import _bounds
from tests._problems import KIND_OF, init_constrained, make_problem

pytestmark = pytest.mark.gpu

LOSS_RTOL = 1e-5
GRAD_RTOL = 1e-4      # tensor rel-L2 per site against the fp64 oracle (BASELINE north_star: 1e-4 relative)


def _shard(kind, kw, z, **extra):
    from scdna_replication_tools_amd.engine import PertShard
    sh = PertShard(KIND_OF[kind], init=init_constrained(kind, z), device="cuda", dirichlet_mode="exact",
                   **kw, **extra)
    sh.set_unconstrained({k: v.numpy() for k, v in z.items()})
    return sh


def _parity(case, kind, prob, kw, z):
    """Loss within LOSS_RTOL, every gradient element inside its Appendix C bound and every
    site's tensor rel-L2 within GRAD_RTOL of the fp64 oracle; the per-site figures go to
    the parity report (tests/_bounds.write_report)."""
    ref_loss, ref_g = po.loss_and_grads(prob, z)
    loss, g = _shard(kind, kw, z).loss_and_grads()
    rep = {}
    entry = {"kind": kind, "shape": list(prob.reads.shape), "loss_rel": abs(loss - float(ref_loss)) / abs(float(ref_loss)),
             "sites": rep}
    skip = ("expose_pi",) if kind.startswith("step1") else ()          # step-1 pi: the canonical block
    try:
        _bounds.check_all(prob, z, g, ref_g, skip=skip, report=rep)
    finally:
        _bounds.write_report(case, entry)
    assert entry["loss_rel"] <= LOSS_RTOL, (loss, float(ref_loss))
    for name, r in rep.items():
        assert r["rel_l2"] <= GRAD_RTOL, (name, r["rel_l2"])


@pytest.mark.parametrize("prior", ["clone", "composite", "product_composite"])
def test_c3_c4_full_genome_shard_step2(prior):
    prob, kw, z = make_problem("step2", L=5451, N=64, prior=prior, num_reads=1e6, seed=21)
    _parity("c3c4_shard_step2_" + prior, "step2", prob, kw, z)


@pytest.mark.parametrize("kind", ["step1", "step1p", "step3"])
def test_c3_c4_full_genome_shard_steps_1_3(kind):
    prob, kw, z = make_problem(kind, L=5451, N=64, num_reads=1e6, seed=23)
    _parity("c3c4_shard_" + kind, kind, prob, kw, z)


def test_c5_20kb_shard():
    prob, kw, z = make_problem("step2", L=136275, N=8, subdivide=25, num_reads=1e6, seed=22, n_libs=1)
    _parity("c5_shard_step2", "step2", prob, kw, z)


def _c4_full(seed, n=10000):
    from scdna_replication_tools_amd.engine import EtaCodebook
    from scdna_replication_tools_amd.init import init_params
    from scdna_replication_tools_amd.simulator import simulate
    sim = simulate(n_s=n, n_g=3, num_reads=1e6, seed=seed)
    reads = sim.reads_s.astype(np.float32)
    eta = EtaCodebook.from_states(sim.cn_s.astype(np.int64), 1e6, 13)          # g1_clones-style prior
    bm = np.zeros((1, 5), np.float32)
    bm[0, 3] = 0.5
    t_init = np.clip(sim.tau_s, 0.05, 0.95).astype(np.float32)
    libs = np.zeros(n, np.int64)
    init = init_params(2, reads, libs, 1, 13, 4, ploidy=eta.argmax_states().mean(0), t_init=t_init,
                       beta_means=bm, seed=0)
    return sim, reads, eta, bm, t_init, libs, init


def test_c4_full_size_pass_per_cell_and_shared_parity():
    from scdna_replication_tools_amd.engine import EtaCodebook, PertShard
    sim, reads, eta, bm, t_init, libs, init = _c4_full(31)
    L, N = reads.shape
    common = dict(lamb=0.75, beta_means=bm, device="cuda", dirichlet_mode="exact", bins_per_tile=60)
    full = PertShard(2, reads, sim.gc, libs, 1, 13, 4, init, eta=eta, **common)
    cells = np.r_[0:8, 4996:5004, 9992:10000]
    loss, g = full.loss_and_grads(pi_cells=cells)
    # the pass is deterministic: a second launch on the same state gives the same bits (each
    # bin's LDS-DMA copies waited for before they are read)
    loss2, g2 = full.loss_and_grads(pi_cells=cells)
    assert loss2 == loss
    for name in ("expose_rho", "expose_a", "expose_pi", "expose_u"):
        assert np.array_equal(np.asarray(g2[name]), np.asarray(g[name])), name
    cn1, rep1 = full.decode()
    cn2, rep2 = full.decode()
    assert torch.equal(cn1, cn2) and torch.equal(rep1, rep2)
    zc = full.unconstrained(pi_cells=cells)
    # oracle on the sampled cells at the same point (the per-cell sites depend on the shared
    # ones and on their own cells only)
    t64 = lambda a: torch.as_tensor(np.asarray(a, np.float64))
    prob = po.OracleProblem("step2", t64(reads[:, cells]), t64(sim.gc.astype(np.float32)), torch.zeros(len(cells),
                            dtype=torch.long), 1, 13, 4, etas=t64(eta.table[eta.codes[:, cells]]),
                            lamb=t64([np.float32(0.75)]), beta_means=t64(bm), t_init=t64(t_init[cells]))
    z = {k: t64(v[cells] if k in ("expose_u", "expose_betas", "expose_tau") else v) for k, v in zc.items()}
    ref_loss, ref_g = po.loss_and_grads(prob, z)
    A = _bounds.contribution_scale(prob, z)
    rep = {}
    for name in ("expose_u", "expose_betas", "expose_tau"):
        gd, gr = np.asarray(g[name])[cells], ref_g[name].numpy()
        rep[name] = dict(rel_l2=_bounds.rel_l2(gd, gr), **_bounds.floor_stats(gr, _bounds.FLOOR_C * A[name]))
        rep[name]["worst_delta_over_bound"] = _bounds.check(name, gd, gr, _bounds.FLOOR_C * A[name])
    pf = _bounds.pi_floor(prob, z)
    rep["expose_pi"] = dict(rel_l2=_bounds.rel_l2(g["expose_pi"], ref_g["expose_pi"].numpy()),
                            **_bounds.floor_stats(ref_g["expose_pi"].numpy(), pf))
    rep["expose_pi"]["worst_delta_over_bound"] = _bounds.check("expose_pi", g["expose_pi"],
                                                               ref_g["expose_pi"].numpy(), pf)
    # the decode of the sampled cells at the same point: every disagreement a near-tie
    dec = _bounds.decode_mismatches(prob, z, cn1[:, torch.as_tensor(cells, device=cn1.device)],
                                    rep1[:, torch.as_tensor(cells, device=rep1.device)])
    _bounds.write_report("c4_full_size_sampled_cells", {"kind": "step2", "shape": [L, N], "cells": cells.tolist(),
                                                        "sites": rep, "decode": dec})
    assert dec["max_ratio"] <= 1.0, dec
    assert dec["mismatches"] <= 1e-3 * dec["n"], dec
    for name, r in rep.items():
        assert r["rel_l2"] <= GRAD_RTOL, (name, r["rel_l2"])
    # shared sites: the full pass equals the sum of four disjoint shards (cuts on 64-cell
    # wave tiles, same tile length: identical per-tile partials, fp64 re-association only)
    del full
    parts = []
    for i, (a, b) in enumerate([(0, 2496), (2496, 4992), (4992, 7488), (7488, N)]):
        sl = slice(a, b)
        init_s = {k: (np.asarray(v)[sl] if k in ("expose_tau", "expose_u", "expose_betas") else v)
                  for k, v in init.items()}
        sh = PertShard(2, reads[:, sl], sim.gc, libs[sl], 1, 13, 4, init_s,
                       eta=EtaCodebook(np.ascontiguousarray(eta.codes[:, sl]), eta.table), is_root=(i == 0),
                       n_cells_total=N, **common)
        parts.append(sh.loss_and_grads())
        del sh
    for name in ("expose_rho", "expose_a", "expose_beta_stds"):
        tot = sum(np.asarray(p[1][name], np.float64) for p in parts)
        np.testing.assert_allclose(tot, np.asarray(g[name], np.float64), rtol=1e-9, atol=0, err_msg=name)
    np.testing.assert_allclose(sum(p[0] for p in parts), loss, rtol=1e-9)


def test_c4_full_size_step2_fit_recovers_truth():
    """configs[3] at full size: the step-2 fit (g1_clones-style prior, 1,000 iterations at most,
    the reference's stopping rule) decodes the simulated states."""
    from scdna_replication_tools_amd.engine import PertShard
    from scdna_replication_tools_amd.tau_init import guess_times_batched
    sim, reads, eta, bm, _, libs, _ = _c4_full(41)
    from scdna_replication_tools_amd.init import init_params
    t_init = guess_times_batched(reads, eta.argmax_states(), 6, device="cuda")[0]
    init = init_params(2, reads, libs, 1, 13, 4, ploidy=eta.argmax_states().mean(0), t_init=t_init, beta_means=bm,
                       seed=0)
    sh = PertShard(2, reads, sim.gc, libs, 1, 13, 4, init, eta=eta, lamb=0.75, beta_means=bm, device="cuda")
    losses, reason = sh.run_svi(1000, 100, 1e-6)
    cn, rep = sh.decode()
    cn = cn.cpu().numpy()
    rep = rep.cpu().numpy()
    acc_cn = (cn == sim.cn_s).mean()
    acc_rep = (rep == sim.rep_s).mean()
    print("C4 fit: {} iterations (reason {}), cn {:.6f}, rep {:.6f}".format(len(losses), reason, acc_cn, acc_rep))
    assert np.isfinite(losses).all() and losses[-1] < losses[0]
    assert acc_cn >= 0.999 and acc_rep >= 0.995, (acc_cn, acc_rep)
