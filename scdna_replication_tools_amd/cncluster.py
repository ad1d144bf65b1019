"""KMeans + BIC clustering of G1/2 cells when no clone labels are given
(reference scdna_replication_tools/cncluster.py:50-120, called by
infer_scRT.py:129-138 when ``clone_col is None``).

The reference fits ``sklearn.cluster.KMeans(n_clusters=k, init="k-means++")`` for every
k in [min_k, max_k] (scikit-learn 0.24.1: n_init = 10 restarts, best inertia kept; the
fits are unseeded) and keeps the k whose ``compute_bic`` is largest.  Here the restarts of
one k run as one batched tensor program on the fit's device (k-means++ seeding with
sklearn's greedy local trials, then Lloyd iterations with sklearn's stopping rule: max
300, strict label convergence or centre shift <= 1e-4 * mean feature variance), and the
BIC is the reference's formula.  ``backend='sklearn'`` runs the reference's own
estimator on the host instead (used by the tests as the behavioural check).
"""
from __future__ import annotations

import logging
from typing import Optional

import numpy as np
import pandas as pd
import torch

log = logging.getLogger("scdna_replication_tools_amd.cncluster")


def compute_bic(centers: np.ndarray, labels: np.ndarray, X: np.ndarray) -> float:
    """cncluster.py:50-78: BIC of a k-means clustering (spherical Gaussian, pooled variance)."""
    X = np.asarray(X, dtype=np.float64)
    centers = np.asarray(centers, dtype=np.float64)
    n_clusters = centers.shape[0]
    cluster_sizes = np.bincount(labels, minlength=n_clusters)
    N, d = X.shape
    sq = ((X - centers[labels]) ** 2).sum()
    cl_var = (1.0 / (N - n_clusters) / d) * sq
    const_term = 0.5 * n_clusters * np.log(N) * (d + 1)
    with np.errstate(divide="ignore", invalid="ignore"):
        terms = (cluster_sizes * np.log(cluster_sizes) - cluster_sizes * np.log(N)
                 - ((cluster_sizes * d) / 2) * np.log(2 * np.pi * cl_var) - ((cluster_sizes - 1) * d / 2))
    return float(np.sum(terms) - const_term)


def compute_bic_tensor(centers: torch.Tensor, labels: torch.Tensor, X: torch.Tensor) -> float:
    """compute_bic on the tensors' device, fp64 (the same formula; only the order of the sum
    of squares differs from numpy's)."""
    X = X.to(torch.float64)
    centers = centers.to(torch.float64)
    n_clusters = centers.shape[0]
    sizes = torch.bincount(labels, minlength=n_clusters).to(torch.float64)
    N, d = X.shape
    sq = float(((X - centers[labels]) ** 2).sum())
    cl_var = (1.0 / (N - n_clusters) / d) * sq
    const_term = 0.5 * n_clusters * np.log(N) * (d + 1)
    sz = sizes.cpu().numpy()
    with np.errstate(divide="ignore", invalid="ignore"):
        terms = (sz * np.log(sz) - sz * np.log(N) - ((sz * d) / 2) * np.log(2 * np.pi * cl_var) - ((sz - 1) * d / 2))
    return float(np.sum(terms) - const_term)


def _sq_dist(X: torch.Tensor, xx: torch.Tensor, C: torch.Tensor) -> torch.Tensor:
    """||x - c||^2 for every (restart, point, centre): (R, N, k), clamped at 0."""
    cc = (C * C).sum(-1)                                           # (R, k)
    d = xx[None, :, None] - 2.0 * torch.matmul(X[None], C.transpose(1, 2)) + cc[:, None, :]
    return d.clamp_(min=0.0)


def _kmeans_pp(X: torch.Tensor, xx: torch.Tensor, k: int, R: int, gen: torch.Generator) -> torch.Tensor:
    """Greedy k-means++ (sklearn _kmeans_plusplus: 2 + floor(log k) local trials per centre,
    the candidate that most reduces the potential wins), R independent restarts -> (R, k, d)."""
    N, d = X.shape
    dev = X.device
    n_trials = 2 + int(np.log(k))
    first = torch.randint(0, N, (R,), generator=gen, device=dev)
    C = torch.empty((R, k, d), dtype=X.dtype, device=dev)
    C[:, 0] = X[first]
    closest = _sq_dist(X, xx, C[:, :1])[:, :, 0]                   # (R, N)
    ar = torch.arange(R, device=dev)
    for c in range(1, k):
        pot = closest.sum(1)                                       # (R,)
        u = torch.rand((R, n_trials), generator=gen, dtype=X.dtype, device=dev) * pot[:, None]
        cand = torch.searchsorted(torch.cumsum(closest, 1), u).clamp_(max=N - 1)   # (R, T)
        dc = _sq_dist(X, xx, X[cand])                              # (R, N, T)
        dc = torch.minimum(dc, closest[:, :, None])
        best = dc.sum(1).argmin(1)                                 # (R,)
        C[:, c] = X[cand[ar, best]]
        closest = dc[ar, :, best]
    return C


def _lloyd(X: torch.Tensor, xx: torch.Tensor, C: torch.Tensor, tol: float, max_iter: int = 300):
    """Lloyd iterations for R restarts at once; returns (centres, labels, inertia)."""
    R, k, d = C.shape
    N = X.shape[0]
    active = torch.ones(R, dtype=torch.bool, device=X.device)
    labels_old = torch.full((R, N), -1, dtype=torch.long, device=X.device)
    for _ in range(max_iter):
        lab = _sq_dist(X, xx, C).argmin(2)                         # (R, N)
        onehot = torch.zeros((R, k, N), dtype=X.dtype, device=X.device)
        onehot.scatter_(1, lab[:, None, :], 1.0)
        cnt = onehot.sum(2)                                        # (R, k)
        new = torch.matmul(onehot, X) / cnt.clamp(min=1.0)[:, :, None]
        new = torch.where(cnt[:, :, None] > 0, new, C)             # empty clusters keep their centre
        shift = ((new - C) ** 2).sum((1, 2))
        same = (lab == labels_old).all(1)
        upd = active & ~same
        C = torch.where(upd[:, None, None], new, C)
        labels_old = torch.where(active[:, None], lab, labels_old)
        active = upd & ~(shift <= tol)
        if not bool(active.any()):
            break
    dist = _sq_dist(X, xx, C)
    lab = dist.argmin(2)
    inertia = dist.gather(2, lab[:, :, None])[:, :, 0].sum(1)
    return C, lab, inertia


def kmeans_fit(X: np.ndarray, k: int, n_init: int = 10, random_state: int = 0, device=None, max_iter: int = 300):
    """One KMeans(n_clusters=k, init='k-means++', n_init=n_init) fit: (centres, labels, inertia)
    of the restart with the least inertia."""
    dev = torch.device(device) if device is not None else torch.device("cuda" if torch.cuda.is_available() else "cpu")
    C, lab, inertia = _kmeans_fit_tensor(torch.as_tensor(np.asarray(X, dtype=np.float64), device=dev), k, n_init,
                                         random_state, max_iter)
    return C.cpu().numpy(), lab.cpu().numpy(), inertia


def _kmeans_fit_tensor(Xt: torch.Tensor, k: int, n_init: int, random_state: int, max_iter: int = 300, tol=None,
                       xx=None):
    """kmeans_fit on a device tensor: (centres, labels) tensors and the inertia."""
    dev = Xt.device
    if tol is None:
        tol = 1e-4 * float(Xt.var(0, unbiased=False).mean())
    if xx is None:
        xx = (Xt * Xt).sum(1)
    gen = torch.Generator(device=dev)
    gen.manual_seed(int(random_state) * 1000003 + k)
    C0 = _kmeans_pp(Xt, xx, k, n_init, gen)
    C, lab, inertia = _lloyd(Xt, xx, C0, tol, max_iter)
    b = int(inertia.argmin())
    return C[b], lab[b], float(inertia[b])


def kmeans_cluster(cn: pd.DataFrame, min_k: int = 2, max_k: int = 100, n_init: int = 10, random_state: int = 0,
                   backend: str = "device", device=None) -> pd.DataFrame:
    """cncluster.py:81-120: cluster the cells (columns of ``cn``, rows = loci) with KMeans for
    every k in [min_k, max_k] and keep the k with the largest BIC.  Returns a frame with
    columns ``cell_id``, ``cluster_id``."""
    X = np.asarray(cn.T.values, dtype=np.float64)
    ks = range(min_k, min(max_k, X.shape[0] - 1) + 1)
    best = None
    if backend == "device":
        # the matrix goes to the device once; every k's fit and BIC run there
        dev = torch.device(device) if device is not None else torch.device(
            "cuda" if torch.cuda.is_available() else "cpu")
        Xt = torch.as_tensor(X, device=dev)
        tol = 1e-4 * float(Xt.var(0, unbiased=False).mean())
        xx = (Xt * Xt).sum(1)
        for k in ks:
            C, lab, _ = _kmeans_fit_tensor(Xt, k, n_init, random_state, tol=tol, xx=xx)
            bic = compute_bic_tensor(C, lab, Xt)
            log.info("k=%d bic=%.6g", k, bic)
            if best is None or bic > best[0]:              # first maximum, like np.argmax
                best = (bic, k, lab)
        log.info("selected k=%d", best[1])
        return pd.DataFrame({"cell_id": cn.columns, "cluster_id": best[2].cpu().numpy()})
    for k in ks:
        if backend == "sklearn":
            import sklearn.cluster
            model = sklearn.cluster.KMeans(n_clusters=k, init="k-means++", n_init=n_init,
                                           random_state=random_state).fit(X)
            centers, labels = model.cluster_centers_, model.labels_
        elif backend == "device":
            centers, labels, _ = kmeans_fit(X, k, n_init=n_init, random_state=random_state, device=device)
        else:
            raise ValueError(backend)
        bic = compute_bic(centers, labels, X)
        log.info("k=%d bic=%.6g", k, bic)
        if best is None or bic > best[0]:                  # first maximum, like np.argmax
            best = (bic, k, labels)
    log.info("selected k=%d", best[1])
    return pd.DataFrame({"cell_id": cn.columns, "cluster_id": best[2]})
