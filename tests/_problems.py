"""Seeded test problems shared by the CPU and GPU parity suites (test infrastructure).

Each builder returns the same problem twice: as an ``oracle.pert_oracle.OracleProblem``
(fp64 reference restatement) and as the keyword arguments of
``scdna_replication_tools_amd.engine.PertShard`` (the device path), plus explicit
unconstrained parameters z so both sides are evaluated at the same point.
"""
from __future__ import annotations

import numpy as np
import torch

from oracle import pert_oracle as po
from scdna_replication_tools_amd.engine import EtaCodebook
from scdna_replication_tools_amd.simulator import simulate

KIND_OF = {"step1": 1, "step2": 2, "step3": 3, "step1p": 1}     # step1p: step 1 in pair mode


def composite_etas(states_a, states_b, P, rng):
    """Composite-style rows (pert_model.py:349-359): 1 + w*J*2 at the clone state plus
    w*(J-j) at the j-th matched G1 cell's state (w = 1e5, J = 5)."""
    L, N = states_a.shape
    e = np.ones((L, N, P), np.float32)
    J, w = 5, 1e5
    np.put_along_axis(e, states_a[..., None], e[np.arange(L)[:, None], np.arange(N)[None, :], states_a][..., None]
                      + w * J * 2, axis=2)
    for j in range(J):
        sj = np.where(rng.uniform(size=(L, N)) < 0.2, states_b, states_a)
        cur = np.take_along_axis(e, sj[..., None], axis=2)
        np.put_along_axis(e, sj[..., None], cur + w * (J - j), axis=2)
    return e


def make_problem(kind: str, L: int = 40, N: int = 70, P: int = 13, K: int = 4, n_libs: int = 2,
                 seed: int = 0, prior: str = "clone", z_scale: float = 1.0, low_reads: bool = False,
                 reads_fn=None, num_reads=None, subdivide: int = 1, pair: bool = False):
    """``L`` bins of the 500 kb grid (or of its ``subdivide``-fold split), ``N`` cells;
    ``num_reads`` per cell (default: a deep 20x coverage of the 500 kb scDNA regime).
    ``pair`` (step 1): the product's training set, N / 2 G1/2 cells doubled with rep 0 / 1
    (pert_model.py:228-251) -- the oracle gets the doubled arrays, PertShard the stored
    half in pair mode (also ``kind="step1p"``)."""
    if kind == "step1p":
        kind, pair = "step1", True
    rng = np.random.default_rng(seed)
    if num_reads is None:
        num_reads = 2e4 if low_reads else 1e6 * L / 5451 * 20
    sim = simulate(n_s=N, n_g=N, n_bins=L, seed=seed, num_reads=num_reads, subdivide=subdivide)
    reads = sim.reads_s.astype(np.float64) if kind != "step1" else sim.reads_g.astype(np.float64)
    if reads_fn is not None:                          # edge cases: all-zero, huge counts
        reads = np.asarray(reads_fn(reads), dtype=np.float64)
    states = (sim.cn_s if kind != "step1" else sim.cn_g).astype(np.int64)
    states = np.minimum(states, P - 1)
    gc = sim.gc.astype(np.float32).astype(np.float64)
    libs = rng.integers(0, n_libs, size=N)
    libs[:n_libs] = np.arange(n_libs)
    product_eta = None
    if prior == "product_composite":
        # the reference's default prior as the PRODUCT builds it: the simulated tables (G1/2 state
        # calls off the clone profile at 2 % of the bins) through pert_infer_scRT's prep --
        # pivots, consensus clone profiles, per-cell Pearson matches, J = 5 composite rows
        # (pert_model.py:299-361) -- and its eta code book; reads, gc and libraries are taken
        # from the same prep (its cell / locus order)
        from scdna_replication_tools_amd import prep
        from scdna_replication_tools_amd.pert_model import pert_infer_scRT
        from scdna_replication_tools_amd.simulator import to_long_form
        assert kind in ("step2", "step3")
        flip = rng.random(sim.cn_g.shape) < 0.02
        sim.cn_g[:] = np.where(flip, np.clip(sim.cn_g + np.where(rng.random(sim.cn_g.shape) < 0.5, -1, 1), 0, P - 1),
                               sim.cn_g)
        df_s, df_g = to_long_form(sim, n_libs=n_libs)
        m = pert_infer_scRT(df_s, df_g, cn_prior_method="g1_composite", device="cpu", log_steps=False)
        inp = m._prepare()
        product_eta = m._build_etas(inp, prep.consensus_clone_profiles(m.cn_g1, m.cn_state_col, keys=inp.keys_g))
        reads = inp.reads_s.astype(np.float64)
        gc = np.asarray(inp.gc, np.float32).astype(np.float64)
        libs = np.asarray(inp.libs_s)
        n_libs = int(libs.max()) + 1
        states = product_eta.argmax_states().astype(np.int64)
    K1 = K + 1
    t64 = lambda a: torch.tensor(np.asarray(a), dtype=torch.float64)

    kw = dict(reads=reads, gc=gc, libs=libs, n_libs=n_libs, P=P, K=K)
    op = dict(kind=kind, reads=t64(reads), gc=t64(gc), libs=torch.tensor(libs, dtype=torch.long),
              n_libs=n_libs, P=P, K=K)
    if kind == "step1":
        rep = np.zeros((L, N))
        rep[:, N // 2:] = 1.0
        if pair:
            assert N % 2 == 0
            half = N // 2
            reads = np.concatenate([reads[:, :half], reads[:, :half]], axis=1)
            states = np.concatenate([states[:, :half], states[:, :half]], axis=1)
            kw.update(reads=reads[:, :half], cn_obs=states[:, :half], paired=True)
            op.update(reads=t64(reads))
        else:
            kw.update(cn_obs=states, rep_obs=rep)
        op.update(cn_obs=t64(states), rep_obs=t64(rep))
    else:
        if product_eta is not None:
            etas = product_eta.dense().astype(np.float32)
        elif prior == "clone":
            etas = np.ones((L, N, P), np.float32)
            np.put_along_axis(etas, states[..., None], 1e6, axis=2)
        elif prior == "composite":
            alt = np.clip(states + rng.integers(-1, 2, size=states.shape), 0, P - 1)
            etas = composite_etas(states, alt, P, rng)
        elif prior == "uniform":
            etas = np.full((L, N, P), 1.0 / P, np.float32)
        else:
            raise ValueError(prior)
        lam = np.float32(0.75)
        bm = (rng.normal(size=(n_libs, K1)) * 0.05).astype(np.float32)
        bm[:, K - 1] += 0.5
        kw.update(eta=product_eta if product_eta is not None else EtaCodebook.from_dense(etas), lamb=float(lam),
                  beta_means=bm)
        op.update(etas=t64(etas), lamb=t64([lam]), beta_means=t64(bm),
                  t_init=t64(np.clip(sim.tau_s, 0.05, 0.95)))
        if kind == "step3":
            rho_f = np.clip(sim.rho_true, 0.02, 0.98).astype(np.float32)
            kw.update(rho_fixed=rho_f, a_fixed=float(np.float32(9.0)))
            op.update(rho_fixed=t64(rho_f).reshape(L, 1), a_fixed=t64([np.float32(9.0)]))
    prob = po.OracleProblem(**op)

    # explicit unconstrained point: a sensible init plus noise (exercises every gradient path)
    if kind != "step1":
        prob_init = prob
    else:
        prob_init = prob
    c = {}
    mu_u = reads.mean(0) / ((1 + 0.5) * 2.0)
    if kind != "step3":
        c["expose_a"] = torch.tensor([8.0 + rng.uniform()], dtype=torch.float64)
        c["expose_rho"] = t64(np.clip(sim.rho_true + rng.normal(size=L) * 0.1, 0.05, 0.95)).reshape(L, 1)
    if kind == "step1":
        c["expose_lambda"] = t64([0.3 + 0.4 * rng.uniform()])
        c["expose_beta_means"] = t64(rng.normal(size=(n_libs, K1)) * 0.1)
    c["expose_beta_stds"] = t64(np.exp(rng.normal(size=(n_libs, K1)) * 0.3) * np.logspace(0, -K, K1)[None, :])
    c["expose_tau"] = t64(rng.uniform(0.1, 0.9, size=N))
    c["expose_u"] = t64(mu_u * (1 + 0.1 * rng.normal(size=N)))
    bet = rng.normal(size=(N, K1)) * 0.05
    bet[:, K - 1] += 0.5
    c["expose_betas"] = t64(bet)
    if kind == "step1":
        pi = np.full((L, N, P), 1.0 / P)
    else:
        zz = rng.normal(size=(L, N, P)) * z_scale
        np.put_along_axis(zz, states[..., None], np.take_along_axis(zz, states[..., None], 2) + 4.0, axis=2)
        pi = np.exp(zz - zz.max(-1, keepdims=True))
        pi /= pi.sum(-1, keepdims=True)
    c["expose_pi"] = t64(pi)
    z = po.unconstrain(kind, c)
    z = {k: v.to(torch.float32).to(torch.float64) for k, v in z.items()}   # representable in fp32
    return prob, kw, z


def init_constrained(kind: str, z):
    """Constrained values of z for PertShard(init=...)."""
    c = po.constrain("step1" if kind == "step1p" else kind, z)
    return {k: v.detach().numpy() for k, v in c.items()}
