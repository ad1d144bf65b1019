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

Arithmetic is fp64 while sklearn fits the profile in its own fp32 arithmetic, and read
counts are integers, so standardised profiles hold many identical values: a group of
them lying on a k-means decision boundary, an EM lower-bound change at the 1e-3
tolerance, a mean gap or skew at its threshold, or a near-tie in the threshold scan
can make the two arithmetics take different branches.  Every such decision is checked
against a margin (``FRAGILE``, relative) and the cells where any of them falls inside
it ("fragile" cells) are recomputed with the reference's per-cell sklearn path
(prep.manhattan_binarization).  Up to ``MINOR_EXACT_MAX_L`` (2,000) bins that covers every
flagged cell (a few %), so the result is the reference's for every cell.  At genome scale
(5,451 bins) the finer near-ties -- a k-means++ draw next to a cumulative-sum boundary, a
threshold scan whose minimum is flat against fp32 summation noise, points within the
levels' rounding budget of the threshold -- flag about half the cells and each per-cell fit
takes about a second, so only the branch decisions are recomputed there and the
near-tie cells keep the batched value.  tests/test_tau_init.py pins both regimes.
"""
from __future__ import annotations

import os

import numpy as np
import torch

MEAN_GAP_THRESH = 0.7
EARLY_S_SKEW_THRESH = 0.2
LATE_S_SKEW_THRESH = -0.2
# Margins of the decisions fp32 (sklearn) vs fp64 (here) rounding could flip: each is a few
# times the rounding difference of the quantity compared (validated on simulated profiles:
# every cell whose batched result differs from the per-cell sklearn one is flagged).  The
# GMM means sklearn's fp32 EM returns carry ~2e-7 sqrt(L) of rounding (1.5e-6 at 271 bins,
# 1.4e-5 at 5,451), which moves the scan's levels and thresholds by as much.
FRAGILE = 1e-5          # relative: mean-gap / skew thresholds
PP_MARGIN = 2e-6        # relative to the k-means++ potential: candidate draw and choice
TIE = 1e-6              # relative width of an exact tie on a k-means decision
EM_MARGIN = 2e-6        # absolute: the EM lower-bound change around its tolerance
MINOR_EXACT_MAX_L = 2000  # up to this many bins, the finer near-ties are recomputed too


EPS32 = float(np.finfo(np.float32).eps)


def _level_margin(L: int) -> float:
    """Relative rounding budget of the scan levels b0, b1 (see above)."""
    return 6e-7 * float(np.sqrt(L))


def _rng_draws(n: int):
    """The data-independent RandomState(0) draws of sklearn's k-means++ for 2 clusters:
    the first centre index and the two local-trial uniforms."""
    rs = np.random.RandomState(0)
    w = np.ones(n, dtype=np.float32)
    first = int(rs.choice(n, p=w / w.sum()))
    u = rs.uniform(size=2 + int(np.log(2)))
    return first, u


def _kmeans_pp(X: torch.Tensor, first: int, u: np.ndarray, fragile: torch.Tensor = None) -> torch.Tensor:
    """k-means++ for 2 centres, batched over the columns of X (L, N) -> (2, N).  Marks in
    ``fragile`` the columns whose candidate draw or choice is within the rounding margin."""
    L, N = X.shape
    c0 = X[first]                                                    # (N,)
    d0 = (X - c0) ** 2                                               # closest_dist_sq (L, N)
    pot = d0.sum(0)                                                  # current_pot
    cums = torch.cumsum(d0, 0)                                       # stable_cumsum
    rv = torch.as_tensor(u, dtype=X.dtype, device=X.device)[:, None] * pot[None, :]     # (T, N)
    cand = torch.searchsorted(cums.T.contiguous(), rv.T.contiguous()).clamp_(max=L - 1)  # (N, T)
    xc = torch.gather(X.T, 1, cand)                                  # (N, T) candidate values
    dist_c = torch.minimum(d0[None, :, :], (X[None, :, :] - xc.T[:, None, :]) ** 2)      # (T, L, N)
    pots = dist_c.sum(1)                                             # (T, N)
    best = pots.argmin(0)                                            # first minimum (N,)
    c1 = xc.gather(1, best[:, None])[:, 0]
    if fragile is not None:
        near = (cums.T.gather(1, cand) - rv.T).abs() <= PP_MARGIN * pot[:, None]
        prev = cums.T.gather(1, (cand - 1).clamp(min=0))
        near |= ((prev - rv.T).abs() <= PP_MARGIN * pot[:, None]) & (cand > 0)
        fragile |= near.any(1)
        differ = (xc[:, 0] != xc[:, 1]) & ((pots[0] - pots[1]).abs() <= PP_MARGIN * pots.abs().max(0).values)
        fragile |= differ
    return torch.stack([c0, c1])


def _assign(X, c, tie_bias: float = 0.0):
    """sklearn's label rule: centre 1 where ||c1||^2 - 2 x c1 < ||c0||^2 - 2 x c0.  Points
    within ``tie_bias`` (relative to the magnitude of the compared values) of the
    decision go to centre 1 (bias > 0) or centre 0 (bias < 0): with integer read counts
    whole groups of identical values sit exactly on a decision, where rounding decides."""
    d1 = c[1] ** 2 - 2 * X * c[1]
    d0 = c[0] ** 2 - 2 * X * c[0]
    if tie_bias == 0.0:
        return (d1 < d0).to(torch.int8)
    scale = c[0] ** 2 + c[1] ** 2 + 2 * X.abs() * (c[0].abs() + c[1].abs())
    return (d1 - d0 < tie_bias * scale).to(torch.int8)


def _lloyd(X: torch.Tensor, centers: torch.Tensor, tol: torch.Tensor, max_iter: int = 300,
           fragile: torch.Tensor = None, tie_bias: float = 0.0):
    """Lloyd's k-means for 2 centres, batched; returns the final labels (L, N) bool
    (True = centre 1) after sklearn's stopping rule and final re-assignment."""
    L, N = X.shape
    labels_old = torch.full((L, N), -1, dtype=torch.int8, device=X.device)
    active = torch.ones(N, dtype=torch.bool, device=X.device)
    strict = torch.zeros(N, dtype=torch.bool, device=X.device)
    c = centers.clone()
    if fragile is None:
        fragile = torch.zeros(N, dtype=torch.bool, device=X.device)
    for _ in range(max_iter):
        # pairwise distance as sklearn's chunked kernel ranks it: ||c||^2 - 2 x c
        lab = _assign(X, c, tie_bias)
        w1 = lab.sum(0).to(X.dtype)
        w0 = L - w1
        s1 = (X * lab).sum(0)
        s0 = X.sum(0) - s1
        new = torch.stack([torch.where(w0 > 0, s0 / w0.clamp(min=1), c[0]),
                           torch.where(w1 > 0, s1 / w1.clamp(min=1), c[1])])
        shift = ((new - c) ** 2).sum(0)
        same = (lab == labels_old).all(0)
        fragile |= active & ~same & ((shift - tol).abs() <= FRAGILE * tol)
        c = torch.where(active[None, :], new, c)
        labels_old = torch.where(active[None, :], lab, labels_old)
        strict |= active & same
        active &= ~same & ~(shift <= tol)
        if not bool(active.any()):
            break
    final = _assign(X, c, tie_bias)
    return torch.where(strict[None, :], labels_old, final).bool()


def _gmm_means(X: torch.Tensor, lab1: torch.Tensor, max_iter: int = 100, tol: float = 1e-3,
               reg_covar: float = 1e-6, fragile: torch.Tensor = None) -> torch.Tensor:
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
        if fragile is not None:
            fragile |= active & ((change.abs() - tol).abs() <= EM_MARGIN)
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


def binarization_fraction(Xraw: torch.Tensor, return_fragile: bool = False, return_minor: bool = False):
    """manhattan_binarization (pert_model.py:364-423) for every column of Xraw (L, N);
    returns the replicated fraction per column (and, with ``return_fragile``, the mask of
    the columns whose outcome fp32 rounding could change, see the module doc): the
    pipeline runs twice, with ties on a k-means decision broken towards either centre,
    and a column whose two results differ is fragile too.  ``return_minor`` splits the
    mask in two: branch decisions (Lloyd / EM stopping, mean-gap and skew thresholds, the
    tie-direction runs disagreeing) and near-ties of finer grain (the k-means++ candidate
    draw, a flat minimum of the threshold scan, points within the levels' rounding budget of
    the chosen threshold)."""
    if not return_fragile:
        return _binarize(Xraw, 0.0)[0]
    f_hi, fr_hi, pp_hi, sc_hi, mn_hi = _binarize(Xraw, TIE, with_minor=True)
    f_lo, fr_lo, pp_lo, sc_lo, mn_lo = _binarize(Xraw, -TIE, with_minor=True)
    decisions = fr_hi | fr_lo | (f_hi != f_lo)
    near = pp_hi | pp_lo | sc_hi | sc_lo | (mn_hi > 0) | (mn_lo > 0)
    if return_minor:
        return f_hi, decisions, near
    return f_hi, decisions | near


def _binarize(Xraw: torch.Tensor, tie_bias: float, with_minor: bool = False):
    X = Xraw.to(torch.float64)
    L, N = X.shape
    X = (X - X.mean(0)) / X.std(0, unbiased=False)
    first, u = _rng_draws(L)
    Xc = X - X.mean(0)                                               # KMeans centres the data first
    tol = Xc.var(0, unbiased=False) * 1e-4
    fragile = torch.zeros(N, dtype=torch.bool, device=X.device)
    frag_pp = torch.zeros(N, dtype=torch.bool, device=X.device)
    frag_scan = torch.zeros(N, dtype=torch.bool, device=X.device)
    lab1 = _lloyd(Xc, _kmeans_pp(Xc, first, u, frag_pp), tol, fragile=fragile, tie_bias=tie_bias)
    mu = _gmm_means(X, lab1, fragile=fragile)
    gap = (mu[0] - mu[1]).abs()
    b0, b1 = torch.minimum(mu[0], mu[1]), torch.maximum(mu[0], mu[1])
    close = gap < MEAN_GAP_THRESH
    fragile |= (gap - MEAN_GAP_THRESH).abs() <= FRAGILE
    if bool(close.any()):
        m2 = (Xc ** 2).mean(0)
        m3 = (Xc ** 3).mean(0)
        skew = m3 / m2 ** 1.5
        fragile |= close & (((skew - EARLY_S_SKEW_THRESH).abs() <= FRAGILE) |
                            ((skew - LATE_S_SKEW_THRESH).abs() <= FRAGILE))
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
    minor = torch.zeros(N, dtype=X.dtype, device=X.device)
    chunk = max(1, int(2e8 // (100 * max(L, 1))))
    for s in range(0, N, chunk):
        xs = X[:, s:s + chunk]
        t = th[:, s:s + chunk]
        hi = xs[None] > t[:, None, :]                                # (100, L, n)
        d = torch.where(hi, (xs[None] - b1[None, None, s:s + chunk]).abs(),
                        (xs[None] - b0[None, None, s:s + chunk]).abs()).sum(1)     # (100, n)
        bi = d.argmin(0)
        best[s:s + chunk] = t.gather(0, bi[None])[0]                 # first minimum
        # a near-tie with a threshold that binarises differently, or a point on the threshold
        # Could the reference pick another threshold?  Its levels differ from these by <= db,
        # which moves every threshold by <= db and changes d(t) - d(t') only through the points
        # t and t' binarise differently (<= 2 db each); a point within ~2 db of a threshold may
        # sit on the other side of it there (changing that d by <= |b1 - b0|); and the
        # reference sums d in fp32 (pairwise: ~eps32 log2(L) relative).
        cnt = hi.sum(1)                                              # (100, n)
        dmin = d.gather(0, bi[None])
        dcnt = (cnt - cnt.gather(0, bi[None])).abs().to(d.dtype)
        db = _level_margin(L) * torch.maximum(b0.abs(), b1.abs())[s:s + chunk]
        span = (b1 - b0)[s:s + chunk].abs()
        near = ((xs[None] - t[:, None, :]).abs() <= 2 * db[None, None] + 1e-6).sum(1).to(d.dtype)   # (100, n)
        near_best = near.gather(0, bi[None])
        slack = (2 * dcnt * db[None] + (near + near_best) * span[None]
                 + 4 * EPS32 * (np.log2(max(L, 2)) + 2) * dmin)
        frag_scan[s:s + chunk] |= (((dcnt > 0) | (near > 0)) & (d - dmin <= slack)).any(0)
        minor[s:s + chunk] = near_best[0]
    frac = (X > best[None, :]).sum(0).to(torch.float64) / L
    if with_minor:
        return frac, fragile, frag_pp, frag_scan, minor
    return frac, fragile | frag_pp | frag_scan | (minor > 0)


def _pool_size(n_jobs: int) -> int:
    return n_jobs if n_jobs > 0 else min(16, len(os.sched_getaffinity(0)))


_WARM = {}


def _warm_worker():
    import sklearn.mixture  # noqa: F401  (the per-cell path's import, done once per worker)
    return 0


def prewarm_pool(n_jobs: int = -1):
    """Start the joblib (loky) worker processes of the per-cell path in a background thread,
    so their start-up (a few seconds: interpreter + sklearn import per worker) overlaps the
    host prep and the first fits instead of delaying guess_times; guess_times_batched waits
    for it and reuses the same executor."""
    import threading
    nj = _pool_size(n_jobs)
    if nj <= 1 or nj in _WARM:
        return

    def run():
        from joblib import Parallel, delayed
        Parallel(n_jobs=nj)(delayed(_warm_worker)() for _ in range(nj))

    th = threading.Thread(target=run, name="pert-tau-pool", daemon=True)
    _WARM[nj] = th
    th.start()


def _pool_state(n_jobs: int) -> str:
    """'none' (no background start), 'warming' or 'ready' -- without waiting."""
    th = _WARM.get(_pool_size(n_jobs))
    if th is None:
        return "none"
    return "warming" if th.is_alive() else "ready"


def guess_times_batched(reads: np.ndarray, cn_states: np.ndarray, upsilon: float = 6, device=None,
                        n_jobs: int = -1):
    """pert_model.py:426-457: (t_init, t_alpha_prior, t_beta_prior), all cells at once; the
    fragile cells (module doc) through the reference's per-cell path, on ``n_jobs``
    processes (-1: the affinity cores, at most 16) when there are many."""
    dev = torch.device(device) if device is not None else torch.device("cpu")
    x = torch.as_tensor(np.asarray(reads, np.float32), device=dev)
    st = torch.as_tensor(np.asarray(cn_states, np.float32), device=dev)
    norm = x / torch.where(st > 0.0, st, torch.full_like(st, 0.5))  # fp32, as the reference divides
    frac, decisions, near = binarization_fraction(norm, return_fragile=True, return_minor=True)
    t = frac.to(torch.float32).cpu().numpy()
    L = norm.shape[0]
    # Up to MINOR_EXACT_MAX_L bins every flagged cell goes through the reference's per-cell
    # path (the result is the reference's).  Above, the finer near-ties are common (half the
    # cells at 5,451 bins: the scan's minimum is flat against fp32 summation noise there, so
    # the reference's own choice is not stable across BLAS builds either) and each per-cell
    # fit takes about a second, so only the branch decisions are recomputed; the cells kept
    # are counted in guess_times_batched.last_near_kept.
    fragile = decisions | near if L <= MINOR_EXACT_MAX_L else decisions
    guess_times_batched.last_near_kept = 0 if L <= MINOR_EXACT_MAX_L else int((near & ~decisions).sum())
    redo = np.flatnonzero(fragile.cpu().numpy())
    if redo.size:
        from .prep import manhattan_binarization
        cols = norm[:, torch.as_tensor(redo, device=dev)].cpu().numpy()
        jobs = [cols[:, j].reshape(-1, 1) for j in range(redo.size)]
        # worker processes only where the per-cell fits outweigh their start-up: more than 64
        # genome-scale cells' worth of bins, or a few cells once the pool is already warm
        state = _pool_state(n_jobs)
        big = redo.size * L > 64 * 5451
        if n_jobs != 1 and redo.size > 4 and (big or state == "ready"):
            if state == "warming":
                _WARM[_pool_size(n_jobs)].join()    # never two executors being built at once
            from joblib import Parallel, delayed
            res = Parallel(n_jobs=_pool_size(n_jobs))(delayed(manhattan_binarization)(c) for c in jobs)
        else:
            res = [manhattan_binarization(c) for c in jobs]
        for j, n in enumerate(redo):
            t[n] = np.float32(res[j][1])
    guess_times_batched.last_fragile = redo
    alpha = (t * np.float32(upsilon)).astype(np.float32)
    return t, alpha, (np.float32(upsilon) - alpha).astype(np.float32)
