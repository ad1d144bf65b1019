"""Batched ``guess_times`` (reference pert_model.py:364-457): the per-cell S-phase time
guess t_init, for every cell at once on the fit's device.

The reference loops over cells in Python and, per cell, standardises the
CN-normalised read profile, fits ``sklearn.mixture.GaussianMixture(n_components=2,
random_state=0)`` (k-means++ / Lloyd initialisation, then EM), picks two binary
levels from the GMM means (or from percentiles chosen by the skew when the means are
closer than 0.7), scans 100 thresholds for the smallest Manhattan distance between
the profile and its binarisation, and returns the replicated fraction.  Here every
stage runs as one batched tensor program over the (L, N) matrix with a per-cell
"still iterating" mask, following the same algorithm and stopping rules:

* k-means++ (sklearn cluster/_kmeans.py ``_kmeans_plusplus``) with the RandomState(0)
  draws sklearn makes - the first-centre ``choice`` and the two local-trial
  ``uniform`` values do not depend on the data, so they are drawn once on the host
  with the same generator and shared by every cell;
* Lloyd iterations (``_kmeans_single_lloyd``: max 300, strict-label or
  centre-shift <= 1e-4 * var convergence, final re-assignment);
* EM of a 2-component 1-D Gaussian mixture (``BaseMixture.fit_predict``: max 100,
  |delta mean log-likelihood| < 1e-3, reg_covar 1e-6, 10 eps on the counts);
* skew (scipy ``skew``, biased), linear percentiles, the 100-threshold scan with
  first-minimum ties.

Arithmetic is fp64 (sklearn runs the fit in the profile's fp32), so a cell whose
scan minimum is a near tie can land one threshold away; tests/test_tau_init.py pins
the agreement with the per-cell sklearn restatement (``prep.manhattan_binarization``).
"""
from __future__ import annotations

import numpy as np
import torch

MEAN_GAP_THRESH = 0.7
EARLY_S_SKEW_THRESH = 0.2
LATE_S_SKEW_THRESH = -0.2


def _rng_draws(n: int):
    """The data-independent RandomState(0) draws of sklearn's k-means++ for 2 clusters:
    the first centre index and the two local-trial uniforms."""
    rs = np.random.RandomState(0)
    w = np.ones(n, dtype=np.float32)
    first = int(rs.choice(n, p=w / w.sum()))
    u = rs.uniform(size=2 + int(np.log(2)))
    return first, u


def _kmeans_pp(X: torch.Tensor, first: int, u: np.ndarray) -> torch.Tensor:
    """k-means++ for 2 centres, batched over the columns of X (L, N) -> (2, N)."""
    L, N = X.shape
    c0 = X[first]                                                    # (N,)
    d0 = (X - c0) ** 2                                               # closest_dist_sq (L, N)
    pot = d0.sum(0)                                                  # current_pot
    cums = torch.cumsum(d0, 0)                                       # stable_cumsum
    rv = torch.as_tensor(u, dtype=X.dtype, device=X.device)[:, None] * pot[None, :]     # (T, N)
    cand = torch.searchsorted(cums.T.contiguous(), rv.T.contiguous()).clamp_(max=L - 1)  # (N, T)
    xc = torch.gather(X.T, 1, cand)                                  # (N, T) candidate values
    dist_c = torch.minimum(d0[None, :, :], (X[None, :, :] - xc.T[:, None, :]) ** 2)      # (T, L, N)
    best = dist_c.sum(1).argmin(0)                                   # first minimum (N,)
    c1 = xc.gather(1, best[:, None])[:, 0]
    return torch.stack([c0, c1])


def _lloyd(X: torch.Tensor, centers: torch.Tensor, tol: torch.Tensor, max_iter: int = 300):
    """Lloyd's k-means for 2 centres, batched; returns the final labels (L, N) bool
    (True = centre 1) after sklearn's stopping rule and final re-assignment."""
    L, N = X.shape
    labels_old = torch.full((L, N), -1, dtype=torch.int8, device=X.device)
    active = torch.ones(N, dtype=torch.bool, device=X.device)
    strict = torch.zeros(N, dtype=torch.bool, device=X.device)
    c = centers.clone()
    for _ in range(max_iter):
        # pairwise distance as sklearn's chunked kernel ranks it: ||c||^2 - 2 x c, ties to centre 0
        lab = ((c[1] ** 2 - 2 * X * c[1]) < (c[0] ** 2 - 2 * X * c[0])).to(torch.int8)
        w1 = lab.sum(0).to(X.dtype)
        w0 = L - w1
        s1 = (X * lab).sum(0)
        s0 = X.sum(0) - s1
        new = torch.stack([torch.where(w0 > 0, s0 / w0.clamp(min=1), c[0]),
                           torch.where(w1 > 0, s1 / w1.clamp(min=1), c[1])])
        shift = ((new - c) ** 2).sum(0)
        same = (lab == labels_old).all(0)
        c = torch.where(active[None, :], new, c)
        labels_old = torch.where(active[None, :], lab, labels_old)
        strict |= active & same
        active &= ~same & ~(shift <= tol)
        if not bool(active.any()):
            break
    final = ((c[1] ** 2 - 2 * X * c[1]) < (c[0] ** 2 - 2 * X * c[0])).to(torch.int8)
    return torch.where(strict[None, :], labels_old, final).bool()


def _gmm_means(X: torch.Tensor, lab1: torch.Tensor, max_iter: int = 100, tol: float = 1e-3,
               reg_covar: float = 1e-6) -> torch.Tensor:
    """EM of a 2-component 1-D GaussianMixture from the k-means labels; (2, N) means."""
    L, N = X.shape
    eps10 = 10 * torch.finfo(X.dtype).eps
    r1 = lab1.to(X.dtype)
    resp = torch.stack([1 - r1, r1])                                 # (2, L, N)

    def m_step(resp):
        nk = resp.sum(1) + eps10                                     # (2, N)
        mu = (resp * X[None]).sum(1) / nk
        var = (resp * (X[None] - mu[:, None, :]) ** 2).sum(1) / nk + reg_covar
        return nk / L, mu, var

    w, mu, var = m_step(resp)
    w = w / w.sum(0, keepdim=True)
    lb = torch.full((N,), -float("inf"), dtype=X.dtype, device=X.device)
    active = torch.ones(N, dtype=torch.bool, device=X.device)
    log2pi = float(np.log(2 * np.pi))
    for _ in range(max_iter):
        prec = var.rsqrt()
        y = (X[None] - mu[:, None, :]) * prec[:, None, :]
        wlp = -0.5 * (log2pi + y * y) + torch.log(prec)[:, None, :] + torch.log(w)[:, None, :]
        lpn = torch.logsumexp(wlp, 0)                                # (L, N)
        resp = torch.exp(wlp - lpn[None])
        w2, mu2, var2 = m_step(resp)
        w2 = w2 / w2.sum(0, keepdim=True)
        lb2 = lpn.mean(0)
        a = active[None, :]
        w, mu, var = torch.where(a, w2, w), torch.where(a, mu2, mu), torch.where(a, var2, var)
        change = lb2 - lb
        lb = torch.where(active, lb2, lb)
        active &= ~(change.abs() < tol)
        if not bool(active.any()):
            break
    return mu


def _percentiles(X: torch.Tensor, qs) -> torch.Tensor:
    """np.percentile(X, 100 q, axis=0) for each q (numpy's 'linear' method, including its
    two-sided lerp), by one column sort; (len(qs), N)."""
    s, _ = torch.sort(X, dim=0)
    L = X.shape[0]
    out = []
    for q in qs:
        pos = q * (L - 1)
        lo = int(np.floor(pos))
        hi = min(lo + 1, L - 1)
        t = pos - lo
        a, b = s[lo], s[hi]
        d = b - a
        out.append(b - d * (1 - t) if t >= 0.5 else a + d * t)
    return torch.stack(out)


def binarization_fraction(Xraw: torch.Tensor) -> torch.Tensor:
    """manhattan_binarization (pert_model.py:364-423) for every column of Xraw (L, N);
    returns the replicated fraction per column."""
    X = Xraw.to(torch.float64)
    L, N = X.shape
    X = (X - X.mean(0)) / X.std(0, unbiased=False)
    first, u = _rng_draws(L)
    Xc = X - X.mean(0)                                               # KMeans centres the data first
    tol = Xc.var(0, unbiased=False) * 1e-4
    lab1 = _lloyd(Xc, _kmeans_pp(Xc, first, u), tol)
    mu = _gmm_means(X, lab1)
    gap = (mu[0] - mu[1]).abs()
    b0, b1 = torch.minimum(mu[0], mu[1]), torch.maximum(mu[0], mu[1])
    close = gap < MEAN_GAP_THRESH
    if bool(close.any()):
        m2 = (Xc ** 2).mean(0)
        m3 = (Xc ** 3).mean(0)
        skew = m3 / m2 ** 1.5
        early = close & (skew > EARLY_S_SKEW_THRESH)
        late = close & ~early & (skew < LATE_S_SKEW_THRESH)
        mid = close & ~early & ~late
        qs = _percentiles(X, [0.05, 0.25, 0.5, 0.75, 0.95])
        b0 = torch.where(early, qs[2], torch.where(late, qs[0], torch.where(mid, qs[1], b0)))
        b1 = torch.where(early, qs[4], torch.where(late, qs[2], torch.where(mid, qs[3], b1)))
    # np.linspace(b0, b1, 100): b0 + i * step, last point exactly b1
    i = torch.arange(100, dtype=X.dtype, device=X.device)[:, None]
    th = b0[None, :] + i * ((b1 - b0) / 99)[None, :]
    th[-1] = b1
    best = torch.empty(N, dtype=X.dtype, device=X.device)
    chunk = max(1, int(2e8 // (100 * max(L, 1))))
    for s in range(0, N, chunk):
        xs = X[:, s:s + chunk]
        t = th[:, s:s + chunk]
        hi = xs[None] > t[:, None, :]                                # (100, L, n)
        d = torch.where(hi, (xs[None] - b1[None, None, s:s + chunk]).abs(),
                        (xs[None] - b0[None, None, s:s + chunk]).abs()).sum(1)     # (100, n)
        best[s:s + chunk] = t.gather(0, d.argmin(0)[None])[0]        # first minimum
    return (X > best[None, :]).sum(0).to(torch.float64) / L


def guess_times_batched(reads: np.ndarray, cn_states: np.ndarray, upsilon: float = 6, device=None):
    """pert_model.py:426-457: (t_init, t_alpha_prior, t_beta_prior), all cells at once."""
    dev = torch.device(device) if device is not None else torch.device("cpu")
    x = torch.as_tensor(np.asarray(reads, np.float32), device=dev)
    st = torch.as_tensor(np.asarray(cn_states, np.float32), device=dev)
    norm = x / torch.where(st > 0.0, st, torch.full_like(st, 0.5))  # fp32, as the reference divides
    t = binarization_fraction(norm).to(torch.float32).cpu().numpy()
    alpha = (t * np.float32(upsilon)).astype(np.float32)
    return t, alpha, (np.float32(upsilon) - alpha).astype(np.float32)
