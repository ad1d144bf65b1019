"""AutoDelta initial values for the three PERT fits (pert_model.py:732, :792, :859).

Pyro's AutoDelta runs the model once under ``init_to_median(num_samples=15)``
(SURVEY.md Appendix B.4): each univariate latent takes the median of 15 draws from
its prior, evaluated in model order with earlier sites at their initial values;
the multivariate Dirichlet site (expose_pi) falls back to a feasible point, which
``transform_to(simplex)`` maps to the uniform simplex; ``pyro.param`` sites start
at their declared init (lambda 0.1 :557, beta_stds logspace(0, -K) :561, tau =
t_init :583).  The draws here come from a ``numpy`` generator seeded with ``seed``
(same distribution as Pyro's init, not the same random stream);
``method="median"`` uses the analytic medians instead (the num_samples -> inf
limit, fully deterministic).
"""
from __future__ import annotations

from typing import Dict, Optional

import numpy as np
from scipy import special, stats


def _median15(rng: np.random.Generator, ppf, shape):
    """The median of 15 draws of the distribution with quantile function ``ppf``: the median
    of an odd number of values is one of them and a quantile function is non-decreasing, so
    median(ppf(u)) = ppf(median(u)) -- one ppf per site instead of 15 (the same values: the
    beta / gamma / normal quantiles over 4 x 200 k draws, bit for bit)."""
    u = rng.uniform(1e-12, 1 - 1e-12, size=(15,) + tuple(shape))
    return ppf(np.median(u, axis=0))


def init_params(kind: int, reads: Optional[np.ndarray], libs: np.ndarray, n_libs: int, P: int, K: int, *,
                ploidy: Optional[np.ndarray] = None, t_init: Optional[np.ndarray] = None,
                beta_means: Optional[np.ndarray] = None, seed: int = 0, method: str = "sampled",
                mean_reads: Optional[np.ndarray] = None, n_bins: Optional[int] = None,
                cells: Optional[slice] = None) -> Dict[str, np.ndarray]:
    """Constrained initial site values (float64) keyed by the reference's site names.
    ``reads`` (L, N) may be replaced by its per-cell means ``mean_reads`` (N,) and ``n_bins``
    (the values are the same; step 1's doubled cells need not be materialised).

    ``cells``: a contiguous range of the N cells (one rank's shard): the per-cell entries
    (tau, u, betas) are returned for those cells only, ``ploidy`` / ``t_init`` /
    ``mean_reads`` are given for them only, and the draws are the ones the whole fit makes
    for them (the generator still draws for all N cells, so a shard's values do not depend
    on the number of ranks)."""
    if mean_reads is None:
        L, N = reads.shape
        src = reads if cells is None else reads[:, cells]
        mean_reads = np.mean(src, axis=0, dtype=np.float64)      # = reads.astype(float64).mean(0), no copy
    else:
        L, N = int(n_bins), int(np.asarray(mean_reads).shape[0])
        if cells is not None:
            N = int(np.asarray(libs).shape[0])
    sl = slice(0, N) if cells is None else cells
    K1 = K + 1
    rng = np.random.default_rng(seed)
    sampled = method == "sampled"
    out: Dict[str, np.ndarray] = {}
    if kind != 3:
        a_med = special.gammaincinv(2.0, 0.5) / 0.2
        out["expose_a"] = (np.array([_median15(rng, lambda u: stats.gamma.ppf(u, 2.0, scale=5.0), (1,))[0]])
                           if sampled else np.array([a_med]))
    if kind == 1:
        out["expose_lambda"] = np.array([0.1])
        out["expose_beta_means"] = (_median15(rng, stats.norm.ppf, (n_libs, K1)) if sampled
                                    else np.zeros((n_libs, K1)))
    out["expose_beta_stds"] = np.tile(np.logspace(0, -K, K1)[None, :], (n_libs, 1))
    if kind != 3:
        out["expose_rho"] = (_median15(rng, lambda u: u, (L,)) if sampled else np.full(L, 0.5))
    if kind == 1:
        tau = (_median15(rng, lambda u: stats.beta.ppf(u, 1.5, 1.5), (N,)) if sampled else np.full(N, 0.5))[sl]
        ploidy = np.full(tau.shape[0], 2.0)
    else:
        tau = np.asarray(t_init, dtype=np.float64)
    out["expose_tau"] = tau
    mu = np.asarray(mean_reads, dtype=np.float64) / ((1 + tau) * np.asarray(ploidy, dtype=np.float64))
    out["expose_u"] = (mu + (mu / 10.0) * _median15(rng, stats.norm.ppf, (N,))[sl]) if sampled else mu
    bm = out["expose_beta_means"] if kind == 1 else np.asarray(beta_means, dtype=np.float64).reshape(n_libs, K1)
    bs = out["expose_beta_stds"]
    libs = np.asarray(libs)[sl]
    loc, scale = bm[libs], bs[libs]
    out["expose_betas"] = (loc + scale * _median15(rng, stats.norm.ppf, (N, K1))[sl]) if sampled else loc.copy()
    return out
