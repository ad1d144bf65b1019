"""Batched ``guess_times`` (reference pert_model.py:364-457): the per-cell S-phase time
guess t_init, for every cell, equal to the reference's per-cell result.

The reference loops over cells in Python and, per cell, standardises the
CN-normalised read profile, fits ``sklearn.mixture.GaussianMixture(n_components=2,
random_state=0)`` (k-means++ / Lloyd initialisation, then EM), picks two binary
levels from the GMM means (or from percentiles chosen by the skew when the means are
closer than 0.7), scans 100 thresholds for the smallest Manhattan distance between
the profile and its binarisation, and returns the replicated fraction -- all in fp32.

Two passes:

* **Batched, fp64, on the fit's device** (``binarization_fraction``): every stage as one
  tensor program over the (L, N) matrix with a per-cell "still iterating" mask --
  k-means++ (sklearn cluster/_kmeans.py ``_kmeans_plusplus``, with the RandomState(0)
  draws sklearn makes, which do not depend on the data), Lloyd (``_kmeans_single_lloyd``:
  max 300, strict-label or centre-shift convergence, final re-assignment), EM of a
  2-component 1-D mixture (``BaseMixture.fit_predict``: max 100, |delta lower bound| <
  1e-3), skew, percentiles, the threshold scan.  Each decision fp32 rounding could flip
  is checked against a margin: the k-means partition (ties of identical read values on
  a decision, a k-means++ draw next to a cumulative-sum boundary, the Lloyd / EM
  stopping rules, the mean-gap and skew thresholds, the two tie-direction runs
  disagreeing) and the scan (a minimum flat against fp32 summation noise, points within
  the levels' rounding budget of the chosen threshold).  A cell none of them flags
  keeps this pass's result.
* **Exact, on the host** (``exact_fractions``) for the flagged cells (a few % up to
  ~2,000 bins, about half at 5,451): the reference's fp32 arithmetic restated call for
  call -- the per-cell standardisation, sklearn's own k-means functions where the
  partition was uncertain (the batched labels otherwise), sklearn's EM op for op with
  the same per-cell BLAS calls, and the scan with the candidate thresholds summed in
  fp32 exactly as ``cityblock`` sums them -- batched over cells where numpy gives the
  same bits, on threads of this process (no worker processes).

So every cell's t_init is bit-identical to the reference's per-cell path
(prep.guess_times) on the same machine; tests/test_tau_init.py checks each stage of the
exact path against sklearn and the whole against prep.guess_times, up to 5,451 bins.
"""
from __future__ import annotations

import contextlib
import os
import threading
import time

import numpy as np
import torch
# the per-cell reference path's modules, imported with this one (as pert_model.py:18-20
# imports them): the exact host path calls them
from scipy.stats import skew
from sklearn.cluster import KMeans


def _private_lloyd():
    """sklearn's own Lloyd iteration (cluster/_kmeans.py ``_kmeans_single_lloyd``), unwrapped,
    or None when this sklearn does not have it with the signature used here.

    It is a private function, so it is only taken after checking its parameters; otherwise
    ``exact_kmeans_labels`` runs the public ``KMeans(...).fit`` call GaussianMixture itself
    makes (same labels, ~1 ms more per cell).  sklearn wraps the function in a threadpoolctl
    limit of 1 BLAS thread (utils/parallel.py _threadpool_controller_decorator) that sets and
    restores OpenBLAS's thread count around every call; entered from several threads at once
    those calls race each other and the other threads' BLAS calls (a 10k-cell run
    deadlocked), so the unwrapped function is called.  Its BLAS work (gemm of a 256-sample
    chunk by 2 one-feature centres) is below OpenBLAS's threading threshold: one thread
    either way, same labels."""
    import inspect
    try:
        from sklearn.cluster._kmeans import _kmeans_single_lloyd as f
    except ImportError:
        return None
    f = getattr(f, "__wrapped__", f)
    try:
        names = list(inspect.signature(f).parameters)
    except (TypeError, ValueError):
        return None
    want = ["X", "sample_weight", "centers_init", "max_iter", "verbose", "tol", "n_threads"]
    return f if names[:len(want)] == want else None


_lloyd_unwrapped = _private_lloyd()
# the public fallback enters threadpoolctl on every call: one caller at a time
_KMEANS_LOCK = threading.Lock()


def _sklearn_threadpool_controller():
    """sklearn's process-wide threadpoolctl controller (utils/parallel.py
    ``_get_threadpool_controller``, created by its first caller), or None."""
    try:
        from sklearn.utils.parallel import _get_threadpool_controller
    except ImportError:
        return None
    return _get_threadpool_controller()


def prepare_host_threads():
    """Make, on the calling thread, every scan of the process's loaded libraries that the
    tau initialiser would otherwise make later from a helper thread; returns sklearn's
    controller (or None).

    threadpoolctl finds the BLAS / OpenMP libraries with ``dl_iterate_phdr`` and a ctypes
    Python callback: the dynamic loader's lock is held while the callback waits for the
    GIL.  A thread that holds the GIL and loads a library at that moment -- an extension
    module import, or a ``ctypes.PyDLL`` call (libpert_hip's launch entry points) whose
    HIP runtime call dlopens -- waits for the loader's lock, and neither thread moves
    again (tools/dl_deadlock_repro.py reproduces it on the CPU within seconds).  The two
    scans are ``_HostHelper``'s search for numpy's BLAS and the creation of sklearn's
    controller (the GaussianMixture / KMeans fallback paths); both are made once per
    process, so after this call no thread of a fit makes one."""
    _HostHelper.get()
    return _sklearn_threadpool_controller()


@contextlib.contextmanager
def host_threads():
    """The fit's host-thread discipline, entered on the fit thread before its helper thread
    starts and left after the helper has ended: the library scans made now
    (``prepare_host_threads``) and, when the public KMeans fallback is in use, the BLAS
    libraries held at one thread for the whole fit -- sklearn's per-call limit then sets
    the thread count to the value it already has instead of raising OpenBLAS's pool again
    while another thread of the fit is inside a BLAS call."""
    ctl = prepare_host_threads()
    if _lloyd_unwrapped is None and ctl is not None:
        with ctl.limit(limits=1, user_api="blas"):
            yield
    else:
        yield


def _tolerance(X: np.ndarray, tol: float) -> float:
    """sklearn cluster/_kmeans.py ``_tolerance`` for dense X: mean of the per-feature
    variances times tol."""
    if tol == 0:
        return 0
    return np.mean(np.var(X, axis=0)) * tol

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
SYNC_EVERY = 4            # batched loops: iterations between host checks for the end


EPS32 = float(np.finfo(np.float32).eps)


def _level_margin(L: int) -> float:
    """Relative rounding budget of the scan levels b0, b1: sklearn's fp32 EM means differ
    from the fp64 ones by up to 4e-7 sqrt(L) of max |mean| (measured against the exact
    restatement, exact_gmm_means, at 271 and 5,451 bins); 2.5x that."""
    return 1e-6 * float(np.sqrt(L))


def _rng_draws(n: int):
    """The data-independent RandomState(0) draws of sklearn's k-means++ for 2 clusters:
    the first centre index and the two local-trial uniforms."""
    rs = np.random.RandomState(0)
    w = np.ones(n, dtype=np.float32)
    first = int(rs.choice(n, p=w / w.sum()))
    u = rs.uniform(size=2 + int(np.log(2)))
    return first, u


def _kmeans_pp(X: torch.Tensor, first: int, u: np.ndarray, fragile: torch.Tensor = None, alts: list = None):
    """k-means++ for 2 centres, batched over the columns of X (L, N) -> (2, N).  Marks in
    ``fragile`` the columns whose candidate draw or choice is within the rounding margin
    and appends to ``alts`` the (N, 6) second centres the reference could have drawn there
    (either trial's candidate and its neighbours on the cumulative sum)."""
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
        if alts is not None:
            nb = torch.cat([(cand - 1).clamp(min=0), cand, (cand + 1).clamp(max=L - 1)], dim=1)   # (N, 6)
            alts.append(torch.gather(X.T, 1, nb))
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
    for it in range(max_iter):
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
        # (finished columns are masked, so iterations past the last one change nothing: the
        # host checks for the end every SYNC_EVERY iterations, not after every one)
        if it % SYNC_EVERY == SYNC_EVERY - 1 and not bool(active.any()):
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
    for it in range(max_iter):
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
        if it % SYNC_EVERY == SYNC_EVERY - 1 and not bool(active.any()):
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
    and a column whose two results (fraction or k-means labels) differ is fragile too.
    ``return_minor`` splits the mask in two -- ``labels``: the k-means partition is not
    certain (Lloyd / EM stopping, mean-gap and skew thresholds, the tie-direction runs
    disagreeing, a k-means++ candidate draw next to a cumulative-sum boundary), and
    ``near``: the partition is certain but the levels' fp32 rounding could move the scan
    (a flat minimum, points within the levels' rounding budget of the chosen threshold) --
    and also returns the (L, N) k-means labels (True = centre 1).

    On a GPU the whole pass of both runs is one launch of the HIP kernel (pert_tau_binarize,
    csrc/tau_kernels.hip); on the CPU it is the tensor programs ``_kmeans_em`` and
    ``_levels_scan`` (the same algorithm, the same margins)."""
    if return_fragile and Xraw.device.type == "cuda":
        hi, lo = binarize_native(Xraw)
        f_hi, fr_hi, pp_hi, sc_hi, mn_hi, lab_hi = hi["frac"], hi["fragile"], hi["pp"], hi["scan"], hi["minor"], hi["labels"]
        f_lo, fr_lo, pp_lo, sc_lo, mn_lo, lab_lo = lo["frac"], lo["fragile"], lo["pp"], lo["scan"], lo["minor"], lo["labels"]
    else:
        X, Xc = _standardize(Xraw)
        if not return_fragile:
            mu, fr, _, _ = _kmeans_em(X, Xc, 0.0)
            return _levels_scan(X, Xc, mu, fr)[0]
        mu_hi, fr_hi, pp_hi, lab_hi = _kmeans_em(X, Xc, TIE)
        mu_lo, fr_lo, pp_lo, lab_lo = _kmeans_em(X, Xc, -TIE)
        f_hi, fr_hi, sc_hi, mn_hi = _levels_scan(X, Xc, mu_hi, fr_hi)
        f_lo, fr_lo, sc_lo, mn_lo = _levels_scan(X, Xc, mu_lo, fr_lo)
    labels = fr_hi | fr_lo | (f_hi != f_lo) | pp_hi | pp_lo | (lab_hi != lab_lo).any(0)
    near = sc_hi | sc_lo | (mn_hi > 0) | (mn_lo > 0)
    if return_minor:
        return f_hi, labels, near, lab_hi
    return f_hi, labels | near


def _standardize(Xraw: torch.Tensor):
    """(X - mean) / std per column in fp64 (pert_model.py:367), and X centred again (KMeans
    centres its data first)."""
    X = Xraw.to(torch.float64)
    X = (X - X.mean(0)) / X.std(0, unbiased=False)
    return X, X - X.mean(0)


def _kmeans_em(X: torch.Tensor, Xc: torch.Tensor, tie_bias: float):
    """The k-means / EM stage as one tensor program over the columns: k-means++ (with the
    alternative second centres where a draw sits on a rounding boundary), Lloyd, EM.
    Returns (GMM means (2, N), fragile (N,), k-means++ fragile (N,), labels (L, N) bool)."""
    L, N = X.shape
    first, u = _rng_draws(L)
    tol = Xc.var(0, unbiased=False) * 1e-4
    fragile = torch.zeros(N, dtype=torch.bool, device=X.device)
    frag_pp = torch.zeros(N, dtype=torch.bool, device=X.device)
    alts = []
    cen = _kmeans_pp(Xc, first, u, frag_pp, alts)
    lab1 = _lloyd(Xc, cen, tol, fragile=fragile, tie_bias=tie_bias)
    if bool(frag_pp.any()):
        # a k-means++ draw within rounding of a boundary: the partition is still certain when
        # Lloyd ends in the same labels from every second centre the reference could have drawn
        idx = torch.nonzero(frag_pp)[:, 0]
        same = torch.ones(idx.numel(), dtype=torch.bool, device=X.device)
        for a in range(alts[0].shape[1]):
            fr_a = torch.zeros(idx.numel(), dtype=torch.bool, device=X.device)
            lab_a = _lloyd(Xc[:, idx], torch.stack([cen[0, idx], alts[0][idx, a]]), tol[idx], fragile=fr_a,
                           tie_bias=tie_bias)
            same &= (lab_a == lab1[:, idx]).all(0) & ~fr_a
        frag_pp[idx[same]] = False
    mu = _gmm_means(X, lab1, fragile=fragile)
    return mu, fragile, frag_pp, lab1


QS = (0.05, 0.25, 0.5, 0.75, 0.95)          # the percentiles the levels may take (pert_model.py:388-399)


def tau_params(L: int):
    """The pert_tau_params of the batched pass at L bins (the constants of this module and the
    sklearn / numpy defaults the reference runs)."""
    from ._native import PertTauParams
    first, u = _rng_draws(L)
    p = PertTauParams()
    p.first, p.lloyd_max_iter, p.em_max_iter = first, 300, 100
    for j, q in enumerate(QS):                       # as _percentiles computes them
        pos = q * (L - 1)
        lo = int(np.floor(pos))
        p.q_lo[j], p.q_hi[j], p.q_t[j] = lo, min(lo + 1, L - 1), pos - lo
    p.u[0], p.u[1] = float(u[0]), float(u[1])
    p.tie, p.pp_margin, p.fragile, p.em_margin = TIE, PP_MARGIN, FRAGILE, EM_MARGIN
    p.em_tol, p.reg_covar = 1e-3, 1e-6
    p.mean_gap, p.early_skew, p.late_skew = MEAN_GAP_THRESH, EARLY_S_SKEW_THRESH, LATE_S_SKEW_THRESH
    p.fragile_abs, p.level_margin, p.eps32 = FRAGILE, _level_margin(L), EPS32
    return p


def binarize_native(Xraw: torch.Tensor):
    """The whole batched pass of both tie directions in ONE launch of pert_tau_binarize (HIP,
    csrc/tau_kernels.hip) on Xraw's device and current stream: per run (tie +TIE, then -TIE)
    a dict of the GMM means (2, N), the k-means labels (L, N) bool, the flags (fragile:
    Lloyd / EM / mean-gap / skew margins; pp: a k-means++ draw; scan: the threshold scan's
    slack), the replicated fraction and the scan's near-threshold count -- what ``_kmeans_em``
    followed by ``_levels_scan`` compute as tensor programs."""
    import ctypes
    from . import _native
    L, N = Xraw.shape
    dev = Xraw.device
    norm = Xraw.to(torch.float32).T.contiguous()                     # (N, L): one row per cell
    labels = torch.empty((2, N, L), dtype=torch.int8, device=dev)
    scratch = torch.empty((2, N, L), dtype=torch.int8, device=dev)
    means = torch.empty((2, N, 2), dtype=torch.float64, device=dev)
    flags = torch.empty((2, N), dtype=torch.int32, device=dev)
    frac = torch.empty((2, N), dtype=torch.float64, device=dev)
    minor = torch.empty((2, N), dtype=torch.float64, device=dev)
    p = tau_params(L)
    stream = torch.cuda.current_stream(dev).cuda_stream
    _native.check(_native.lib().pert_tau_binarize(L, N, norm.data_ptr(), ctypes.byref(p), labels.data_ptr(),
                                                  scratch.data_ptr(), means.data_ptr(), flags.data_ptr(),
                                                  frac.data_ptr(), minor.data_ptr(), ctypes.c_void_p(stream)),
                  "pert_tau_binarize")
    return [dict(mu=means[r].T, labels=labels[r].T.bool(), fragile=(flags[r] & 1) != 0, pp=(flags[r] & 2) != 0,
                 scan=(flags[r] & 4) != 0, frac=frac[r], minor=minor[r]) for r in range(2)]


def _levels_scan(X: torch.Tensor, Xc: torch.Tensor, mu: torch.Tensor, fragile: torch.Tensor):
    """The levels (GMM means, or percentiles chosen by the skew when the means are close)
    and the 100-threshold scan (pert_model.py:375-423) for every column, with the rounding
    margins of the scan.  Returns (fraction, fragile, scan fragile, minor)."""
    L, N = X.shape
    fragile = fragile.clone()
    frag_scan = torch.zeros(N, dtype=torch.bool, device=X.device)
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
        # fp32 summation: the reference's d(t) and d(t') are pairwise sums of the same terms
        # except at the dcnt points t and t' binarise differently, so every partial sum of the
        # tree away from those points is bitwise the same in both and cancels; what remains is
        # the rounding along the paths from those points to the root -- at most u |partial|
        # per node: <= (16 + 16 + 3 x 8) x 16 terms of the point's leaf block (numpy's 8
        # accumulators of <= 16 terms, three combining levels) and d / 2^h at tree level h
        # (min(2^h, dcnt) such nodes) -- in each of the two sums.
        tmax = torch.maximum((xs - b0[None, s:s + chunk]).abs(), (xs - b1[None, s:s + chunk]).abs()).amax(0)
        noise = EPS32 * (dcnt * 56 * 16 * tmax[None] + (torch.log2(dcnt + 1) + 2) * dmin)
        # a point x within 2 db of a threshold may sit on its other side in the reference: that
        # moves d by |x - b1| - |x - b0| = b0 + b1 - 2x (x between the levels), i.e. by at most
        # |b0 + b1 - 2t| + 4 db -- small near the scan's optimum, the levels' midpoint
        mid = (b0 + b1)[None, s:s + chunk]
        flip = (mid - 2 * t).abs() + 4 * db[None]
        slack = 2 * dcnt * db[None] + near * flip + near_best * flip.gather(0, bi[None]) + noise
        frag_scan[s:s + chunk] |= (((dcnt > 0) | (near > 0)) & (d - dmin <= slack)).any(0)
        minor[s:s + chunk] = near_best[0]
    frac = (X > best[None, :]).sum(0).to(torch.float64) / L
    return frac, fragile, frag_scan, minor


# ------------------------------------------------------------------------------------------
# The exact host path: the reference's per-cell fp32 arithmetic, restated call for call and
# batched over cells where numpy gives the same bits (elementwise ufuncs, per-row reductions),
# with the same BLAS calls per cell as sklearn makes.  tests/test_tau_init.py checks every
# stage against sklearn / the per-cell reference bit for bit.
F32 = np.float32
_LOG2PI32 = np.log(2 * np.pi).astype(np.float32)        # _estimate_log_gaussian_prob's constant
_EPS10 = 10 * np.finfo(np.float32).eps                   # _estimate_gaussian_parameters' nk guard
_NEG_INF = F32(-np.inf)
SCAN_SLACK = 1e-4   # relative: fp64 scan values within this of the minimum are re-summed in fp32


def standardize_rows(norm_rows: np.ndarray) -> np.ndarray:
    """``(X - np.mean(X)) / np.std(X)`` (pert_model.py:367) for every row of an (n, L) fp32
    array: numpy's per-row reductions are the 1-D ones (pairwise sums), so each row equals
    the reference's per-cell result."""
    X = np.ascontiguousarray(norm_rows, dtype=F32)
    return (X - np.mean(X, axis=1, keepdims=True)) / np.std(X, axis=1, keepdims=True)


def _sq_dist_upcast(c: np.ndarray, X: np.ndarray) -> np.ndarray:
    """sklearn metrics/pairwise.py ``_euclidean_distances(c, X, Y_norm_squared=<fp32>,
    squared=True)`` for fp32 data with one feature: ``_euclidean_distances_upcast`` forms
    -2 c x + c^2 + x^2 in float64 (the product and squares are exact there), casts to
    float32 and clips at 0.  (k, 1), (L, 1) -> (k, L) float32."""
    c64 = c.astype(np.float64)
    x64 = X.astype(np.float64)
    d = -2 * (c64 @ x64.T)
    d += c64 * c64
    d += (x64 * x64).T
    out = d.astype(np.float32)
    np.maximum(out, 0, out=out)
    return out


def exact_kmeans_labels(x: np.ndarray) -> np.ndarray:
    """The labels of ``cluster.KMeans(n_clusters=2, n_init=1, random_state=RandomState(0))
    .fit(X)`` as GaussianMixture's k-means initialisation runs it (sklearn
    mixture/_base.py _initialize_parameters; cluster/_kmeans.py KMeans.fit): tolerance from
    the uncentred data, centring by the fp32 mean, k-means++ (``_kmeans_plusplus`` restated
    with the same RandomState draws, distances and BLAS products), then sklearn's own Lloyd
    (``_kmeans_single_lloyd``, on one OpenMP thread: the reference's thread count only
    changes the last bits of the centre sums, never a label short of an exact tie).  Without
    that function (``_private_lloyd``) the public call itself runs."""
    X = np.array(x, dtype=F32, order="C").reshape(-1, 1)
    if _lloyd_unwrapped is None:
        return public_kmeans_labels(X)
    n = X.shape[0]
    tol = _tolerance(X, 1e-4)
    rs = np.random.RandomState(0)
    sw = np.ones(n, dtype=X.dtype)
    X -= X.mean(axis=0)
    centers = np.empty((2, 1), dtype=X.dtype)
    centers[0] = X[rs.choice(n, p=sw / sw.sum())]
    closest = _sq_dist_upcast(centers[0, np.newaxis], X)
    pot = closest @ sw
    rand_vals = rs.uniform(size=2 + int(np.log(2))) * pot
    cand = np.searchsorted(np.cumsum(sw * closest, dtype=np.float64), rand_vals)
    np.clip(cand, None, closest.size - 1, out=cand)
    dc = _sq_dist_upcast(X[cand], X)
    np.minimum(closest, dc, out=dc)
    centers[1] = X[cand[np.argmin(dc @ sw.reshape(-1, 1))]]
    labels, _, _, _ = _lloyd_unwrapped(X, sw, centers, max_iter=300, verbose=False, tol=tol, n_threads=1)
    return labels.astype(np.int8)


def public_kmeans_labels(x: np.ndarray) -> np.ndarray:
    """GaussianMixture's k-means initialisation through sklearn's public API, the call of
    mixture/_base.py ``_initialize_parameters``: ``KMeans(n_clusters=2, n_init=1,
    random_state=<RandomState(0)>).fit(X).labels_`` (one caller at a time)."""
    X = np.array(x, dtype=F32, order="C").reshape(-1, 1)
    with _KMEANS_LOCK:
        km = KMeans(n_clusters=2, n_init=1, random_state=np.random.RandomState(0)).fit(X)
    return km.labels_.astype(np.int8)


def _lse2(a: np.ndarray) -> np.ndarray:
    """scipy.special.logsumexp(a, axis=-1) of an (..., 2) fp32 array, op for op as scipy's
    _logsumexp (b=None); its two-element reductions written as the equal elementwise ops."""
    a0, a1 = a[..., 0], a[..., 1]
    a_max = np.maximum(a0, a1)
    i0, i1 = a0 == a_max, a1 == a_max
    m = i0.astype(F32) + i1.astype(F32)
    shift = np.where(np.isfinite(a_max), a_max, F32(0))
    am = np.empty_like(a)
    am[..., 0] = np.where(i0, _NEG_INF, a0)
    am[..., 1] = np.where(i1, _NEG_INF, a1)
    with np.errstate(divide="ignore", invalid="ignore", over="ignore", under="ignore"):
        e = np.exp(am - shift[..., None])
        s = e[..., 0] + e[..., 1]
        s = np.where(s == 0, s, s / m)
        sgn = np.sign(s + 1) * np.sign(m)
        s = np.where(s < -1, -s - 2, s)
        out = np.log1p(s) + np.log(np.abs(m)) + a_max
    out[sgn < 0] = np.nan
    return out


class _HostHelper:
    """libpert_host.so (csrc/pert_host.c: the EM's M step and lower bound over all bins, the
    GIL released) bound to numpy's own BLAS (the cblas_sgemv / cblas_sdot numpy calls for
    ``np.dot``).  ``get()`` is None when either is not available; the numpy restatement then
    runs the same operations (same results, slower)."""
    _inst = False
    _lock = threading.Lock()

    @classmethod
    def get(cls):
        # loaded once, under a lock: threadpoolctl's library scan (dl_iterate_phdr) from
        # several of the exact path's threads at once is not safe
        with cls._lock:
            if cls._inst is False:
                cls._inst = cls._load()
        return cls._inst

    @staticmethod
    def _load():
        import ctypes
        from ctypes import POINTER, c_float, c_int64, c_void_p
        path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libpert_host.so")
        blas = _numpy_blas()
        if blas is None or not os.path.exists(path):
            return None
        from . import build as _build
        # a library built from other sources (an ABI or arithmetic change) is not loaded:
        # the numpy restatement runs instead
        if _build.host_embedded_hash(path) != _build.host_source_hash():
            return None
        try:
            lib = ctypes.CDLL(path)                       # CDLL: the calls release the GIL
        except OSError:
            return None
        f = lib.pert_host_em_mstep
        fp = POINTER(c_float)
        f.argtypes = [c_int64, c_int64, c_int64, POINTER(c_int64), fp, fp, POINTER(c_int64), fp, c_void_p, c_void_p,
                      fp, fp, fp, fp, fp]
        f.restype = ctypes.c_int
        lib.pert_host_pairwise_sum.argtypes = [fp, c_int64]
        lib.pert_host_pairwise_sum.restype = c_float
        h = _HostHelper()
        h.lib, h.sgemv, h.sdot = lib, blas[0], blas[1]
        return h

    def mstep(self, rows, resp_u, lpn_u, inv, X):
        """(nk, means, cov + reg_covar, lb) of the cells ``rows`` (see pert_host.c)."""
        import ctypes
        from ctypes import POINTER, c_float, c_int64
        m, U = resp_u.shape[0], resp_u.shape[1]
        L = X.shape[1]
        rows = np.ascontiguousarray(rows, dtype=np.int64)
        resp_u = np.ascontiguousarray(resp_u, dtype=F32)
        nk, means, cov = (np.empty((m, 2), F32) for _ in range(3))
        lb = np.empty(m, F32)
        scratch = np.empty(4 * L, F32)
        fp = lambda a: a.ctypes.data_as(POINTER(c_float))
        lp = None
        if lpn_u is not None:
            lpn_u = np.ascontiguousarray(lpn_u, dtype=F32)
            lp = fp(lpn_u)
        self.lib.pert_host_em_mstep(m, L, U, rows.ctypes.data_as(POINTER(c_int64)), fp(resp_u), lp,
                                    inv.ctypes.data_as(POINTER(c_int64)), fp(X), self.sgemv, self.sdot,
                                    fp(nk), fp(means), fp(cov), fp(lb), fp(scratch))
        return nk, means, cov, lb


def _numpy_blas():
    """Addresses of cblas_sgemv / cblas_sdot in the BLAS numpy itself calls (its bundled
    scipy-openblas, ILP64 interface), or None."""
    import ctypes
    try:
        from threadpoolctl import threadpool_info
        libs = [d for d in threadpool_info() if d.get("user_api") == "blas" and "numpy" in d.get("filepath", "")]
    except Exception:                                     # noqa: BLE001  (no threadpoolctl / odd layout)
        return None
    for d in libs:
        try:
            h = ctypes.CDLL(d["filepath"])
        except OSError:
            continue
        for pre, suf in (("scipy_", "64_"), ("", "64_")):
            try:
                g = getattr(h, pre + "cblas_sgemv" + suf)
                s = getattr(h, pre + "cblas_sdot" + suf)
            except AttributeError:
                continue
            return ctypes.cast(g, ctypes.c_void_p).value, ctypes.cast(s, ctypes.c_void_p).value
    return None


def _distinct(Xs: np.ndarray):
    """Per row of Xs (n, L): the sorted distinct values, their counts and the inverse map."""
    n, L = Xs.shape
    uniq, counts, inv = [], [], np.empty((n, L), np.intp)
    for i in range(n):
        u, iv, c = np.unique(Xs[i], return_inverse=True, return_counts=True)
        uniq.append(u)
        counts.append(c)
        inv[i] = iv
    return uniq, counts, inv


def exact_gmm_means(Xs: np.ndarray, labels: np.ndarray, max_iter: int = 100, tol: float = 1e-3,
                    distinct=None, use_host: bool = True) -> np.ndarray:
    """``GaussianMixture(n_components=2, random_state=0).fit_predict(X).means_`` for every
    row X of Xs (n, L) fp32, from the k-means ``labels`` (n, L): sklearn's EM
    (mixture/_base.py fit_predict; _gaussian_mixture.py _initialize, _m_step,
    _estimate_gaussian_parameters, _estimate_log_gaussian_prob with 'full' covariances, one
    feature) restated op for op.  The E step is elementwise in x, so it runs on each row's
    distinct values and is gathered back.  The M step's sums are the reference's own:
    ``resp.sum(axis=0)`` (numpy adds the rows in order, i.e. a cumulative sum), and per cell
    the BLAS calls sklearn makes -- ``np.dot(resp.T, X)`` (gemv on an (L, 2) C-ordered
    array) and ``np.dot(resp[:, k] * diff.T, diff)`` (sdot of two contiguous vectors); the
    1x1 Cholesky factor and triangular solve are sqrt and 1 / l.  The M step runs in
    libpert_host.so when it and numpy's BLAS are found (``use_host``), else in numpy: the
    same operations either way.  Returns (n, 2) fp32."""
    n, L = Xs.shape
    Xs = np.ascontiguousarray(Xs, dtype=F32)
    host = _HostHelper.get() if use_host else None
    xs = [np.array(Xs[i], dtype=F32).reshape(L, 1) for i in range(n)] if host is None else None
    uniq, _, inv = _distinct(Xs) if distinct is None else distinct
    inv = np.ascontiguousarray(inv, dtype=np.int64)
    U = max(len(u) for u in uniq)
    Xu = np.empty((n, U), F32)
    for i, u in enumerate(uniq):
        Xu[i, :len(u)] = u
        Xu[i, len(u):] = u[0]
    if host is not None:
        # the initial M step through the helper: "distinct values" = the two labels
        lab = np.ascontiguousarray(labels, dtype=np.int64)
        onehot = np.broadcast_to(np.eye(2, dtype=F32)[None], (n, 2, 2))
        w, means, cov, _ = host.mstep(np.arange(n), onehot, None, lab, Xs)
    else:
        resp = np.zeros((n, L, 2), dtype=F32)
        resp[np.arange(n)[:, None], np.arange(L)[None, :], np.asarray(labels, np.intp)] = 1

    def mstep(resp, rows):
        m = len(rows)
        nk = np.cumsum(resp, axis=1)[:, -1, :] + _EPS10                  # (m, 2)
        dots = np.empty((m, 2), F32)
        for j, i in enumerate(rows):
            dots[j] = np.dot(resp[j].copy().T, xs[i])[:, 0]
        means = dots / nk
        diff = Xs[rows][:, None, :] - means[:, :, None]                   # (m, 2, L): X - means[k]
        prod = resp.transpose(0, 2, 1) * diff                             # resp[:, k] * diff.T
        cov = np.empty((m, 2), F32)
        for j in range(m):
            cov[j, 0] = np.dot(prod[j, 0], diff[j, 0])
            cov[j, 1] = np.dot(prod[j, 1], diff[j, 1])
        return nk, means, cov / nk + 1e-6

    if host is None:
        w, means, cov = mstep(resp, np.arange(n))
    w = w / L
    pc = F32(1) / np.sqrt(cov)
    lower = np.full(n, -np.inf, dtype=F32)
    active = np.ones(n, bool)
    for _ in range(max_iter):
        a = np.flatnonzero(active)
        pa = pc[a]
        y = Xu[a][:, :, None] * pa[:, None, :] - (means[a] * pa)[:, None, :]
        wlp = (-0.5 * (1 * _LOG2PI32 + np.square(y)) + np.log(pa)[:, None, :]) + np.log(w[a])[:, None, :]
        lpn_u = _lse2(wlp)
        with np.errstate(under="ignore"):
            resp_u = np.exp(wlp - lpn_u[:, :, None])
        if host is not None:
            w2, m2, c2, lb = host.mstep(a, resp_u, lpn_u, inv, Xs)
        else:
            ia = inv[a] + (np.arange(len(a)) * U)[:, None]   # flat gather of the distinct values
            lb = np.mean(np.take(lpn_u, ia), axis=1)
            ia2 = 2 * ia
            w2, m2, c2 = mstep(np.take(resp_u, np.stack([ia2, ia2 + 1], axis=2)), a)
        w[a] = w2 / (w2[:, :1] + w2[:, 1:])
        means[a], cov[a] = m2, c2
        pc[a] = F32(1) / np.sqrt(c2)
        change = lb - lower[a]
        lower[a] = lb
        active[a[np.abs(change) < tol]] = False
        if not active.any():
            break
    return means


def exact_scan(x: np.ndarray, mean_0, mean_1, MEAN_GAP=MEAN_GAP_THRESH, EARLY=EARLY_S_SKEW_THRESH,
               LATE=LATE_S_SKEW_THRESH, distinct=None) -> float:
    """pert_model.py:377-423 for one standardized fp32 profile x (L,) and the GMM means:
    the levels (means, or percentiles chosen by the skew), ``np.linspace(b0, b1, 100)``
    thresholds and the first threshold of least ``cityblock(X, B)``; returns the replicated
    fraction.  The 100 distances are evaluated in fp64 from sorted prefix sums; only the
    thresholds within SCAN_SLACK of the least are summed the reference's way (fp32
    ``abs(X - B).sum()``; its error is < 1e-5 of the sum), which decides among them."""
    X = np.asarray(x, dtype=F32).reshape(-1)
    L = X.size
    mean_gap = abs(mean_0 - mean_1)
    b0, b1 = min(mean_0, mean_1), max(mean_0, mean_1)
    if mean_gap < MEAN_GAP:
        cs = skew(X)
        if cs > EARLY:
            b0, b1 = np.percentile(X, 50), np.percentile(X, 95)
        elif cs < LATE:
            b0, b1 = np.percentile(X, 5), np.percentile(X, 50)
        else:
            b0, b1 = np.percentile(X, 25), np.percentile(X, 75)
    th = np.linspace(b0, b1, 100)
    u, c = np.unique(X, return_counts=True) if distinct is None else distinct
    u64 = u.astype(np.float64)
    C = np.concatenate([[0], np.cumsum(c)])                  # points among the first j distinct values
    S = np.concatenate([[0.0], np.cumsum(c * u64)])
    nu = len(u64)
    k = np.searchsorted(u64, th.astype(np.float64), side="right")     # x <= t: B = b0 there

    def absdev(lo, hi, level):
        # sum of |x - level| over the distinct-value ranges [lo, hi), split at the level
        m = np.minimum(np.maximum(np.searchsorted(u64, level, side="right"), lo), hi)
        return ((C[m] - C[lo]) * level - (S[m] - S[lo])) + ((S[hi] - S[m]) - (C[hi] - C[m]) * level)

    d = absdev(np.zeros_like(k), k, float(b0)) + absdev(k, np.full_like(k, nu), float(b1))
    cand = np.flatnonzero(d <= d.min() * (1 + SCAN_SLACK) + 1e-9)
    best, lowest = None, np.inf
    for i in cand:                                            # in threshold order, strict '<'
        dist = np.abs(X - np.where(X > th[i], b1, b0)).sum()
        if dist < lowest:
            lowest, best = dist, th[i]
    cell_rt = np.where(X > best, 1, 0)
    return cell_rt.sum() / len(cell_rt)


def exact_fractions(norm_cols: np.ndarray, labels=None, n_threads: int = 1, chunk: int = None) -> np.ndarray:
    """The reference's replicated fraction (manhattan_binarization, pert_model.py:364-423)
    of every column of ``norm_cols`` (L, n) fp32 (the CN-normalised reads), bit for bit:
    standardisation, k-means labels (``labels`` (n, L) where the batched pass has settled
    them, rows of -1 to compute them here), GMM EM, threshold scan.  Runs in this process,
    chunks of cells on ``n_threads`` threads (numpy releases the GIL in the array work)."""
    Xs_all = standardize_rows(np.asarray(norm_cols, dtype=F32).T)
    n = Xs_all.shape[0]
    _HostHelper.get()                       # before the threads start
    out = np.empty(n, np.float64)

    def run(lo, hi):
        Xs = Xs_all[lo:hi]
        lab = np.empty(Xs.shape, np.int8)
        for j in range(hi - lo):
            if labels is None or labels[lo + j][0] < 0:
                lab[j] = exact_kmeans_labels(Xs[j])
            else:
                lab[j] = labels[lo + j]
        dist = _distinct(Xs)
        mu = exact_gmm_means(Xs, lab, distinct=dist)
        for j in range(hi - lo):
            out[lo + j] = exact_scan(Xs[j], mu[j, 0], mu[j, 1], distinct=(dist[0][j], dist[1][j]))

    if chunk is None:
        # large chunks: the EM runs batched over a chunk, and its per-iteration Python work (which
        # holds the GIL the threads share) is paid once per chunk, not once per cell
        chunk = max(32, min(128, -(-n // max(1, n_threads))))
    spans = [(i, min(n, i + chunk)) for i in range(0, n, chunk)]
    if _lloyd_unwrapped is None and (labels is None or np.any(np.asarray(labels)[:, 0] < 0)):
        # the public KMeans fallback sets and restores the BLAS thread count on every call,
        # racing the BLAS calls of the other threads: those cells take one thread
        n_threads = 1
    if n_threads <= 1 or len(spans) == 1:
        for lo, hi in spans:
            run(lo, hi)
    else:
        from concurrent.futures import ThreadPoolExecutor
        with ThreadPoolExecutor(max_workers=min(n_threads, len(spans)), thread_name_prefix="pert-tau") as ex:
            for f in [ex.submit(run, lo, hi) for lo, hi in spans]:
                f.result()
    return out


def default_threads() -> int:
    """Threads of the exact host path: one.  Its per-cell work is short numpy calls that hold
    the GIL, so more threads do not go faster (C4's 1,831 flagged cells on the GPU box: 0.56 s
    on 1 thread, 0.52-0.61 s on 2-16, profiles/r03za_exact_threads.log) and, inside a fit,
    take the GIL from the thread queueing the device's steps (step 1 ran at 0.94 instead of
    0.4 ms/step while 16 of them ran)."""
    return 1


def cn_normalise(reads: np.ndarray, cn_states: np.ndarray) -> np.ndarray:
    """reads / where(state > 0, state, 0.5) in fp32 (pert_model.py:446-448: the states cast to
    float32, each quotient the correctly rounded fp32 division torch performs), by locus tiles
    on a few threads."""
    from concurrent.futures import ThreadPoolExecutor
    x = np.asarray(reads, np.float32)
    st = np.asarray(cn_states)
    if x.shape != st.shape or x.ndim != 2:
        raise ValueError("reads and CN states must be (loci, cells) of one shape")
    out = np.empty(x.shape, np.float32)
    T = 256

    def tile(l0):
        s = st[l0:l0 + T].astype(np.float32)
        np.divide(x[l0:l0 + T], np.where(s > 0.0, s, np.float32(0.5)), out=out[l0:l0 + T])
    with ThreadPoolExecutor(max_workers=8) as ex:
        list(ex.map(tile, range(0, x.shape[0], T)))
    return out


def guess_times_batched(reads: np.ndarray, cn_states: np.ndarray, upsilon: float = 6, device=None,
                        n_threads: int = None):
    """pert_model.py:426-457: (t_init, t_alpha_prior, t_beta_prior), all cells at once.
    The batched fp64 pass (device) decides every cell whose result fp32 rounding cannot
    change; the others take the exact host path (exact_fractions) -- with the batched
    k-means labels where the partition is certain, else with sklearn's own k-means -- so
    every cell's t_init is the reference's.  No worker processes."""
    t0 = time.perf_counter()
    dev = torch.device(device) if device is not None else torch.device("cpu")
    # the reference's normalisation (:446-448), on the host in fp32 (these are the values
    # the exact path standardises); the batched pass reads the same values on the device
    norm = torch.from_numpy(cn_normalise(reads, cn_states))
    frac, lab_unsure, near, lab = binarization_fraction(norm.to(dev), return_fragile=True, return_minor=True)
    t = frac.to(torch.float32).cpu().numpy()
    redo = np.flatnonzero((lab_unsure | near).cpu().numpy())
    t1 = time.perf_counter()
    if redo.size:
        sel = torch.as_tensor(redo, device=lab.device)
        labels = lab[:, sel].T.to(torch.int8).cpu().numpy()
        labels[lab_unsure[sel].cpu().numpy()] = -1            # k-means recomputed on the host
        nt = default_threads() if n_threads is None else int(n_threads)
        fr = exact_fractions(norm[:, torch.as_tensor(redo)].numpy(), labels, n_threads=nt)
        t[redo] = fr.astype(np.float32)
        guess_times_batched.last_kmeans = int((labels[:, 0] < 0).sum())
    else:
        guess_times_batched.last_kmeans = 0
    guess_times_batched.last_fragile = redo
    guess_times_batched.last_timings = {"batched_s": t1 - t0, "exact_s": time.perf_counter() - t1,
                                        "cells": int(norm.shape[1]), "exact_cells": int(redo.size),
                                        "kmeans_cells": guess_times_batched.last_kmeans}
    alpha = (t * np.float32(upsilon)).astype(np.float32)
    return t, alpha, (np.float32(upsilon) - alpha).astype(np.float32)
