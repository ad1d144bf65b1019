"""Elementwise gradient bounds of SURVEY.md Appendix C (test infrastructure).

Every gradient element of the device path must satisfy

    |g_dev - g64| <= RTOL * |g64| + floor

against the fp64 oracle, with RTOL = 1e-4 and the floor

* expose_pi (per bin, cell, state k): 4 eps32 * sum_j (eta_j - 1) * pi_k -- Appendix C's
  term for the Dirichlet softmax-backward, the cancellation fp32 cannot avoid;
* every other site: ``FLOOR_C * A`` where A is the sum of the absolute values of the
  per-(bin, cell) contributions that make up that gradient element (plus its prior
  term): an fp32 pipeline that evaluates each contribution to a relative accuracy e
  and sums them cannot be closer than ~e * A to the exact sum where those contributions
  cancel.  A comes from the oracle itself (``contribution_scale``): the data term is
  differentiated w.r.t. per-(bin, cell) copies of each site, the absolute values summed
  over the reduced axis;

plus, for the enumerated fits (steps 2/3), the responsibility term: the joint scores
s(c, r) are O(x log x) sums an fp32 pipeline holds to ~eps32 * M_s (M_s: the magnitude
of the terms of that score), and an error ds in the scores moves the contribution
sum_s gamma_s b_s (b_s = d s_s / d site) by sum_s gamma_s (ds_s - mean ds) (b_s - mean b):
``SCORE_C * eps32 * sum gamma_s M_s |b_s - b_bar|`` over the reduced axis
(``score_sensitivity``).  At deep coverage (thousands of reads per bin) this dominates:
the reference's own fp32 evaluation (lgamma of O(1e4) arguments) is ten times coarser.
"""
from __future__ import annotations

import numpy as np
import torch

from oracle import pert_oracle as po

RTOL = 1e-4
EPS32 = float(np.finfo(np.float32).eps)
FLOOR_C = 2e-6          # per-contribution accuracy budget of the fp32 device arithmetic
SCORE_C = 4.0           # roundings per score term in the device's fp32 score


def _expand(z: dict, L: int, N: int) -> dict:
    """Per-(bin, cell) leaf copies of the sites the data term reads."""
    ex = {}
    for name, v in z.items():
        v = v.detach()
        if name in ("expose_u", "expose_tau"):
            ex[name] = v.reshape(1, N).expand(L, N).clone()
        elif name == "expose_betas":
            ex[name] = v.reshape(1, N, -1).expand(L, N, v.shape[-1]).clone()
        elif name == "expose_rho":
            ex[name] = v.reshape(L, 1).expand(L, N).clone()
        elif name in ("expose_a", "expose_lambda"):
            ex[name] = v.reshape(1, 1).expand(L, N).clone()
        else:
            ex[name] = v.clone()
        ex[name].requires_grad_(True)
    return ex


def contribution_scale(prob: po.OracleProblem, z: dict) -> dict:
    """A per gradient element (see module doc), fp64, shaped like the gradients."""
    prob = prob.to(torch.float64)
    z = {k: v.to(torch.float64) for k, v in z.items()}
    L, N = prob.reads.shape
    ploidy = po.cell_ploidies(prob)
    # data term per (bin, cell)
    ex = _expand(z, L, N)
    t = po.model_terms(prob, po.constrain(prob.kind, ex), global_terms=False, ploidy=ploidy)
    data = t["enum"] if "enum" in t else t["reads"] + t["rep"]
    data.backward()
    A = {}
    for name, v in ex.items():
        if v.grad is None or name == "expose_pi":
            continue
        g = v.grad.abs()
        if name in ("expose_u", "expose_tau"):
            A[name] = g.sum(0)
        elif name == "expose_betas":
            A[name] = g.sum(0)
        elif name == "expose_rho":
            A[name] = g.sum(1).reshape(L, 1)
        elif name in ("expose_a", "expose_lambda"):
            A[name] = g.sum().reshape(1)
    # prior terms (one contribution per element, added once)
    zz = {k: v.detach().clone().requires_grad_(True) for k, v in z.items()}
    tp = po.model_terms(prob, po.constrain(prob.kind, zz), ploidy=ploidy)
    prior = sum(v for k, v in tp.items() if k not in ("enum", "reads", "rep", "cn", "expose_pi"))
    prior.backward()
    for name, v in zz.items():
        if name == "expose_pi" or v.grad is None:
            continue
        A[name] = A.get(name, torch.zeros_like(v)) + v.grad.abs().reshape(A[name].shape if name in A else v.shape)
    # beta_stds / beta_means: sums over cells of per-cell prior terms
    c = po.constrain(prob.kind, {k: v.detach() for k, v in z.items()})
    bm = c["expose_beta_means"] if prob.kind == "step1" else prob.beta_means.to(torch.float64)
    bs = c["expose_beta_stds"]
    w = (c["expose_betas"] - bm[prob.libs]) / bs[prob.libs]
    per_bs = torch.zeros_like(bs).index_add_(0, prob.libs, (w * w - 1).abs())
    A["expose_beta_stds"] = per_bs
    if prob.kind == "step1":
        A["expose_beta_means"] = torch.zeros_like(bm).index_add_(0, prob.libs, (w / bs[prob.libs]).abs()) + bm.abs()
    return {k: v.detach().numpy() for k, v in A.items()}


def score_magnitudes(prob: po.OracleProblem, z: dict) -> torch.Tensor:
    """M_s (2P, L, N): the magnitude of the terms the device sums into each joint score --
    log pi~, log Bern, delta log(1 - lam), and the NB's (delta - 1/2) log1p(x/delta) and
    x log1p(delta/x) (pert_math.h's asymptotic form)."""
    with torch.no_grad():
        c = po.constrain(prob.kind, z)
        x = prob.reads
        L, N = x.shape
        P = prob.P
        u, betas = c["expose_u"], c["expose_betas"]
        gcf = po.gc_features(prob.gc, prob.K).reshape(L, 1, -1)
        omega = torch.exp((betas * gcf).sum(2))
        lam = prob.lamb
        cn = torch.arange(P, dtype=x.dtype).reshape(P, 1, 1)
        rep = torch.tensor([0., 1.], dtype=x.dtype).reshape(2, 1, 1, 1)
        delta = (u * cn * (1 + rep) * omega * (1 - lam) / lam).clamp(min=1.0)
        xx = x.expand_as(delta)
        nb = (delta * torch.log1p(-lam)).abs() + ((delta - 0.5) * torch.log1p(xx / delta)).abs() \
            + torch.where(xx > 0, xx * torch.log1p(delta / xx.clamp(min=1e-300)), torch.zeros_like(xx)).abs()
        s = po.enum_scores(prob, z).abs()
        return (nb + s).reshape(2 * P, L, N)


def score_sensitivity(prob: po.OracleProblem, z: dict) -> dict:
    """SCORE_C eps32 sum gamma_s M_s |b_s - b_bar| per gradient element (module doc)."""
    prob = prob.to(torch.float64)
    z = {k: v.to(torch.float64) for k, v in z.items()}
    L, N = prob.reads.shape
    P = prob.P
    ex = _expand(z, L, N)
    s = po.enum_scores(prob, ex).reshape(2 * P, L, N)
    gam = torch.softmax(s.detach(), 0)
    M = score_magnitudes(prob, z)
    names = [k for k in ex if tuple(ex[k].shape[:2]) == (L, N)]
    bs = {k: [] for k in names}
    for i in range(2 * P):
        gr = torch.autograd.grad(s[i].sum(), [ex[k] for k in names], retain_graph=True, allow_unused=True)
        for k, g in zip(names, gr):
            bs[k].append(torch.zeros_like(ex[k]) if g is None else g.detach())
    out = {}
    for k in names:
        b = torch.stack(bs[k])                                    # (2P, L, N[, ...]) per state
        gm = gam.reshape((2 * P, L, N) + (1,) * (b.dim() - 3))
        Mm = M.reshape((2 * P, L, N) + (1,) * (b.dim() - 3))
        bbar = (gm * b).sum(0, keepdim=True)
        per = SCORE_C * EPS32 * (gm * Mm * (b - bbar).abs()).sum(0)  # per (bin, cell[, ...])
        if k in ("expose_u", "expose_tau", "expose_betas"):
            out[k] = per.sum(0)
        elif k == "expose_rho":
            out[k] = per.sum(1).reshape(L, 1)
        elif k in ("expose_a", "expose_lambda"):
            out[k] = per.sum().reshape(1)
        elif k == "expose_pi":
            out[k] = per
    return {k: v.numpy() for k, v in out.items()}


def pi_floor(prob: po.OracleProblem, z: dict) -> np.ndarray:
    """Appendix C: 4 eps32 * sum_j (eta_j - 1) * pi_k per (bin, cell, state)."""
    pi = torch.softmax(z["expose_pi"].to(torch.float64), -1)
    S1 = (prob.etas.to(torch.float64) - 1).sum(-1, keepdim=True)
    return (4 * EPS32 * S1.abs() * pi).numpy()


def check(name: str, g_dev, g64, floor) -> float:
    """Largest |delta| / bound over the tensor (<= 1 passes); raises with the worst element."""
    g_dev = np.asarray(g_dev, np.float64).reshape(np.shape(g64))
    g64 = np.asarray(g64, np.float64)
    bound = RTOL * np.abs(g64) + np.broadcast_to(np.asarray(floor, np.float64), g64.shape)
    ratio = np.abs(g_dev - g64) / np.maximum(bound, 1e-300)
    worst = float(ratio.max()) if ratio.size else 0.0
    if worst > 1.0:
        i = np.unravel_index(int(ratio.argmax()), ratio.shape)
        raise AssertionError("{}: |delta| / bound = {:.3g} at {} (dev {:.9g}, fp64 {:.9g}, bound {:.3g})".format(
            name, worst, i, g_dev[i], g64[i], bound[i]))
    return worst


def floor_stats(g64, floor) -> dict:
    """How loose the floor is: floor / |g64| over the elements (median, p99, max) and the
    fraction of elements where the floor, not RTOL |g64|, sets the bound."""
    g = np.abs(np.asarray(g64, np.float64)).reshape(-1)
    f = np.broadcast_to(np.asarray(floor, np.float64), np.shape(g64)).reshape(-1)
    r = f / np.maximum(g, 1e-300)
    return {"floor_over_g64_median": float(np.median(r)), "floor_over_g64_p99": float(np.percentile(r, 99)),
            "floor_over_g64_max": float(r.max()), "floor_dominant_frac": float((f > RTOL * g).mean())}


def check_all(prob: po.OracleProblem, z: dict, g_dev: dict, g64: dict, skip=(), report: dict = None) -> dict:
    """``check`` for every site of g64; returns {site: worst ratio}.  With ``report``, also
    records per site the worst ratio, the tensor rel-L2 error and the floor statistics."""
    A = contribution_scale(prob, z)
    S = score_sensitivity(prob, z) if prob.kind != "step1" else {}
    out = {}
    for name, ref in g64.items():
        if name in skip:
            continue
        ref = ref.detach().numpy() if isinstance(ref, torch.Tensor) else np.asarray(ref)
        floor = pi_floor(prob, z) if name == "expose_pi" else FLOOR_C * A[name].reshape(ref.shape)
        if name in S:
            floor = floor + S[name].reshape(ref.shape)
        if report is not None:
            gd = np.asarray(g_dev[name], np.float64).reshape(ref.shape)
            report[name] = dict(rel_l2=rel_l2(gd, ref), **floor_stats(ref, floor))
        out[name] = check(name, g_dev[name], ref, floor)
        if report is not None:
            report[name]["worst_delta_over_bound"] = out[name]
    return out


def rel_l2(a, b) -> float:
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def write_report(case: str, entry: dict, path: str = None):
    """Merge ``entry`` under ``case`` into the JSON parity report (default
    gpurun_out/parity_report.json, or $PERT_PARITY_REPORT)."""
    import json
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    path = path or os.environ.get("PERT_PARITY_REPORT", os.path.join(root, "gpurun_out", "parity_report.json"))
    os.makedirs(os.path.dirname(path), exist_ok=True)
    data = {}
    if os.path.exists(path):
        try:
            with open(path) as fh:
                data = json.load(fh)
        except ValueError:
            data = {}
    data[case] = entry
    with open(path, "w") as fh:
        json.dump(data, fh, indent=1, sort_keys=True)


def decode_mismatches(prob, z, cn_dev, rep_dev, c: float = 8.0, nb_rel: float = 5e-6) -> dict:
    """Account for every (bin, cell) whose decoded joint state (infer_discrete temperature 0,
    pert_model.py:820-827) differs from the fp64 oracle's joint argmax at the same point.
    Each such disagreement must be a near-tie: the oracle's score gap between its best state
    B and the device's choice A, s(B) - s(A) >= 0, is set against the fp32 error bound of
    the two scores, E(A) + E(B), with

        E = c eps32 (|log pi~| + |log Bern| + |NB'| + delta |d NB'/d delta|) + nb_rel max(1, |NB'|)

    (NB' = the reads term without its state-independent part kappa, the quantity the kernels
    evaluate; nb_rel = the device special functions' accuracy, test_nb_lgdiff_device_accuracy;
    the delta term covers delta's own fp32 rounding).  Returns the counts, the largest
    gap / bound ratio (<= 1 when every mismatch is a near-tie) and the worst cases."""
    from oracle import pert_oracle as po
    eps = float(np.finfo(np.float32).eps)
    with torch.no_grad():
        t = po.enum_score_terms(prob, z)
    P = prob.P
    L, N = prob.reads.shape
    nbp = t["lp_reads"] - t["kappa"]
    E = (c * eps * (t["lp_cn"].abs() + t["lp_rep"].abs() + nbp.abs() + t["delta"] * t["dpsi"].abs())
         + nb_rel * torch.clamp(nbp.abs(), min=1.0))
    s = t["score"].reshape(2 * P, L, N).numpy()
    E = E.reshape(2 * P, L, N).numpy()
    best = np.argmax(s, axis=0)
    cn_dev = np.asarray(cn_dev.cpu() if isinstance(cn_dev, torch.Tensor) else cn_dev).astype(np.int64)
    rep_dev = np.asarray(rep_dev.cpu() if isinstance(rep_dev, torch.Tensor) else rep_dev).astype(np.int64)
    dev = rep_dev * P + cn_dev
    mism = np.argwhere(dev != best)
    out = dict(n=int(L * N), mismatches=int(len(mism)), max_ratio=0.0, worst=[])
    if len(mism):
        li, ni = mism[:, 0], mism[:, 1]
        b, a = best[li, ni], dev[li, ni]
        gap = s[b, li, ni] - s[a, li, ni]
        bound = E[b, li, ni] + E[a, li, ni]
        ratio = gap / bound
        order = np.argsort(-ratio)[:5]
        out["max_ratio"] = float(ratio.max())
        out["worst"] = [dict(bin=int(li[k]), cell=int(ni[k]), oracle_state=int(b[k]), device_state=int(a[k]),
                             gap=float(gap[k]), bound=float(bound[k])) for k in order]
    return out
