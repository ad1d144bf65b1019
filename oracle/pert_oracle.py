"""PERT oracle: CPU restatement of the reference SVI hot path.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module, and only as the
checker (or, for the baseline, as the thing timed on the host CPU).  The product
path (``scdna_replication_tools_amd``) never imports it and has no CPU fallback.

What it restates
----------------
``pert_infer_scRT.model_s`` (reference ``scdna_replication_tools/pert_model.py:541-646``)
as it is fitted by ``run_pert_model`` (``pert_model.py:649-901``):

* step 1 (``:718-774``): ``poutine.condition(model_s, {cn, rep})`` fitted with
  ``JitTrace_ELBO``; latent a, beta_means, rho, tau (Beta(1.5,1.5)), u, betas, pi;
  params lambda, beta_stds.
* step 2 (``:776-830``): cn x rep enumerated (``JitTraceEnum_ELBO(max_plate_nesting=2)``),
  beta_means observed, lambda passed in, tau a ``pyro.param`` initialised at t_init.
* step 3 (``:834-896``): step 2 with rho and a observed (frozen).

Pyro itself (pyro-ppl 1.8.2, ``requirements4.txt:159``) is NOT vendored under
/root/reference and is not importable here.  The
restatement therefore uses the library Pyro wraps for every log density --
``torch.distributions`` (Gamma, Beta, Normal, Dirichlet, Categorical, Bernoulli,
NegativeBinomial, Independent) and ``torch.distributions.transform_to`` for the
AutoDelta / ``pyro.param`` unconstrained storage -- and states the Pyro semantics
it relies on explicitly:

* B.1 enumeration: per (bin, cell) logsumexp over the 2 x P joint (rep, cn) states
  of the summed log factors, then a sum over the plates;
* B.2 AutoDelta guide: Delta log-density 0, so ELBO = log joint at the point;
* B.3 storage: simplex -> SoftmaxTransform, unit_interval -> clipped sigmoid,
  interval -> sigmoid + affine, positive -> exp, real -> identity;
* B.4 init: ``init_to_median(num_samples=15)`` for univariate sites, the
  multivariate Dirichlet site falls back to a feasible point (uniform simplex);
* B.5 optimiser: one ``torch.optim.Adam`` (lr, betas=(0.8, 0.99), eps=1e-8) per param;
* B.6 ``poutine.condition`` does not touch ``pyro.param`` sites, so beta_stds is
  re-initialised and re-learned in steps 2 and 3;
* B.7 ``infer_discrete(temperature=0)`` = per-element joint argmax over (rep, cn).

PARITY UNPINNED: the reference's own tests pin no numbers on this path
(``test_with_pytest.py:70-78`` checks columns only; ``:81-102`` never calls
``infer`` and its data is absent) and the reference cannot be imported here.  The
oracle is pinned instead by (i) using torch.distributions directly, (ii) brute-force
per-element loops and autograd checks in ``tests/test_oracle.py``, and
(iii) ground-truth recovery on simulator data.  See DESIGN.md, "Oracle".
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np
import torch
from torch.distributions import (Bernoulli, Beta, Categorical, Dirichlet, Gamma, Independent,
                                 NegativeBinomial, Normal, constraints, transform_to)

KINDS = ("step1", "step2", "step3")

# Adam hyper-parameters of ``pyro.optim.Adam({'lr': lr, 'betas': [0.8, 0.99]})``
# (pert_model.py:734, :793, :860) on top of torch.optim.Adam defaults (eps=1e-8).
ADAM_BETAS = (0.8, 0.99)
ADAM_EPS = 1e-8


# --------------------------------------------------------------------------- sites
# (name, constraint) of every optimised site, in model execution order.
# pert_model.py:553 (a), :557 (lambda), :560 (beta_means), :561 (beta_stds),
# :574 (rho), :581-585 (tau), :600 (u), :603 (betas), :611 (pi).
_INTERVAL_LAMBDA = constraints.interval(0.001, 0.999)

PARAM_SITES: Dict[str, List[tuple]] = {
    "step1": [("expose_a", constraints.positive),
              ("expose_lambda", _INTERVAL_LAMBDA),
              ("expose_beta_means", constraints.real),
              ("expose_beta_stds", constraints.positive),
              ("expose_rho", constraints.unit_interval),
              ("expose_tau", constraints.unit_interval),
              ("expose_u", constraints.real),
              ("expose_betas", constraints.real),
              ("expose_pi", constraints.simplex)],
    "step2": [("expose_a", constraints.positive),
              ("expose_beta_stds", constraints.positive),
              ("expose_rho", constraints.unit_interval),
              ("expose_tau", constraints.unit_interval),
              ("expose_u", constraints.real),
              ("expose_betas", constraints.real),
              ("expose_pi", constraints.simplex)],
    "step3": [("expose_beta_stds", constraints.positive),
              ("expose_tau", constraints.unit_interval),
              ("expose_u", constraints.real),
              ("expose_betas", constraints.real),
              ("expose_pi", constraints.simplex)],
}


@dataclass
class OracleProblem:
    """Inputs of one SVI fit, in the reference's tensor layout.

    reads (L, N) fp (integer valued, pert_model.py:163-166); gc (L,); libs (N,) int64;
    etas (L, N, P) for steps 2/3; cn_obs / rep_obs (L, N) for step 1;
    lamb (1,) and beta_means (n_libs, K+1) for steps 2/3; rho_fixed (L, 1) and
    a_fixed (1,) for step 3.
    """
    kind: str
    reads: torch.Tensor
    gc: torch.Tensor
    libs: torch.Tensor
    n_libs: int
    P: int = 13
    K: int = 4
    etas: Optional[torch.Tensor] = None
    cn_obs: Optional[torch.Tensor] = None
    rep_obs: Optional[torch.Tensor] = None
    lamb: Optional[torch.Tensor] = None
    beta_means: Optional[torch.Tensor] = None
    rho_fixed: Optional[torch.Tensor] = None
    a_fixed: Optional[torch.Tensor] = None
    t_init: Optional[torch.Tensor] = None

    def __post_init__(self):
        assert self.kind in KINDS, self.kind

    @property
    def shape(self):
        return tuple(self.reads.shape)

    def to(self, dtype) -> "OracleProblem":
        def cv(t):
            if t is None or not torch.is_floating_point(t):
                return t
            return t.to(dtype)
        return OracleProblem(self.kind, cv(self.reads), cv(self.gc), self.libs, self.n_libs,
                             self.P, self.K, cv(self.etas), cv(self.cn_obs), cv(self.rep_obs),
                             cv(self.lamb), cv(self.beta_means), cv(self.rho_fixed),
                             cv(self.a_fixed), cv(self.t_init))

    def cells(self, sl: slice) -> "OracleProblem":
        """Restrict to a contiguous cell range (the cell plate is independent given
        the shared per-bin / global values)."""
        def c2(t):
            return None if t is None else t[:, sl]
        return OracleProblem(self.kind, self.reads[:, sl], self.gc, self.libs[sl], self.n_libs,
                             self.P, self.K,
                             None if self.etas is None else self.etas[:, sl],
                             c2(self.cn_obs), c2(self.rep_obs), self.lamb, self.beta_means,
                             self.rho_fixed, self.a_fixed,
                             None if self.t_init is None else self.t_init[sl])


def gc_features(gc: torch.Tensor, K: int) -> torch.Tensor:
    """pert_model.py:460-463 -- columns [gc^K, ..., gc, 1] (reversed powers)."""
    x = gc.unsqueeze(1)
    return torch.cat([x ** i for i in reversed(range(0, K + 1))], 1)


def constrain(kind: str, z: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    """Unconstrained storage -> constrained site values (B.3, transform_to registry)."""
    out = {}
    for name, con in PARAM_SITES[kind]:
        out[name] = transform_to(con)(z[name])
    return out


def unconstrain(kind: str, c: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    out = {}
    for name, con in PARAM_SITES[kind]:
        out[name] = transform_to(con).inv(c[name])
    return out


def _t(v, like):
    return torch.tensor(v, dtype=like.dtype)


def cell_ploidies(prob: OracleProblem) -> torch.Tensor:
    """pert_model.py:589-595."""
    L, N = prob.reads.shape
    if prob.kind == "step1":
        return torch.ones(N, dtype=prob.reads.dtype) * 2.
    temp_cn0 = torch.argmax(prob.etas, dim=2).type(prob.reads.dtype)
    return torch.mean(temp_cn0, dim=0)


def model_terms(prob: OracleProblem, c: Dict[str, torch.Tensor], *, global_terms: bool = True,
                ploidy: Optional[torch.Tensor] = None) -> Dict[str, torch.Tensor]:
    """Per-site summed log densities of ``model_s`` at the point ``c``.

    Mirrors pert_model.py:541-646 line by line.  For steps 2/3 the enumerated
    sites cn (dim -3) and rep (dim -4) are contracted per plate element by a
    logsumexp over the 2 x P joint states (B.1).  ``global_terms=False`` drops the
    sites outside the cell plate (used when a problem is evaluated in cell chunks).
    """
    kind = prob.kind
    x = prob.reads
    L, N = x.shape
    P, K = prob.P, prob.K
    dt = x.dtype
    terms = {}

    # a ~ Gamma(2, 0.2)  (:553); observed in step 3 (:847)
    a = c["expose_a"] if kind != "step3" else prob.a_fixed
    if global_terms:
        terms["expose_a"] = Gamma(_t([2.], x), _t([0.2], x)).log_prob(a).sum()
    # lambda (:556-557)
    lamb = c["expose_lambda"] if kind == "step1" else prob.lamb
    # beta_means ~ N(0,1)^{n_libs x K+1}  (:560); observed in steps 2/3 (:785)
    bm = c["expose_beta_means"] if kind == "step1" else prob.beta_means
    if global_terms:
        # Pyro's .to_event(n) == torch Independent(d, n)
        terms["expose_beta_means"] = Independent(Normal(_t(0., x), _t(1., x)).expand(
            [prob.n_libs, K + 1]), 2).log_prob(bm)
    bs = c["expose_beta_stds"]                                     # (:561-562)
    # rho ~ Beta(1,1) per bin (:572-574); observed in step 3 (:847)
    rho = c["expose_rho"] if kind != "step3" else prob.rho_fixed
    if global_terms:
        terms["expose_rho"] = Beta(_t([1.], x), _t([1.], x)).log_prob(rho).sum()
    # tau (:580-585)
    tau = c["expose_tau"]
    if kind == "step1":
        terms["expose_tau"] = Beta(_t([1.5], x), _t([1.5], x)).log_prob(tau).sum()
    # u (:589-600)
    if ploidy is None:
        ploidy = cell_ploidies(prob)
    u_guess = torch.mean(x, dim=0) / ((1 + tau) * ploidy)
    u_stdev = u_guess / 10.
    u = c["expose_u"]
    terms["expose_u"] = Normal(u_guess, u_stdev).log_prob(u).sum()
    # betas (:603)
    betas = c["expose_betas"]
    terms["expose_betas"] = Independent(Normal(bm[prob.libs], bs[prob.libs]), 1).log_prob(betas).sum()
    # pi ~ Dirichlet(etas) (:607-611)
    pi = c["expose_pi"]
    etas = torch.ones(L, N, P, dtype=dt) if kind == "step1" else prob.etas
    terms["expose_pi"] = Dirichlet(etas).log_prob(pi).sum()

    # phi (:616-623) -- literal 1/(1+exp(-a t)); clamps zero the gradient
    t_diff = tau.reshape(-1, N) - rho.reshape(L, -1)
    phi = 1 / (1 + torch.exp(-a * t_diff))
    phi = torch.where(phi < 0.001, torch.full_like(phi, 0.001), phi)
    phi = torch.where(phi > 0.999, torch.full_like(phi, 0.999), phi)
    # omega (:632-633)
    gcf = gc_features(prob.gc, K).reshape(L, 1, K + 1)
    omega = torch.exp(torch.sum(torch.mul(betas, gcf), 2))

    if kind == "step1":
        cn = prob.cn_obs
        rep = prob.rep_obs
        terms["cn"] = Categorical(pi).log_prob(cn).sum()
        terms["rep"] = Bernoulli(phi).log_prob(rep).sum()
        chi = cn * (1. + rep)
        theta = u * chi * omega
        delta = theta * (1 - lamb) / lamb
        delta = torch.where(delta < 1, torch.ones_like(delta), delta)
        terms["reads"] = NegativeBinomial(delta, probs=lamb).log_prob(x).sum()
    else:
        cn = torch.arange(P).reshape(P, 1, 1)                     # enum dim -3
        rep = torch.tensor([0., 1.], dtype=dt).reshape(2, 1, 1, 1)  # enum dim -4
        lp_cn = Categorical(pi).log_prob(cn)                      # (P, L, N)
        lp_rep = Bernoulli(phi).log_prob(rep)                     # (2, 1, L, N)
        chi = cn * (1. + rep)                                     # (2, P, 1, 1)
        theta = u * chi * omega
        delta = theta * (1 - lamb) / lamb
        delta = torch.where(delta < 1, torch.ones_like(delta), delta)
        lp_reads = NegativeBinomial(delta, probs=lamb).log_prob(x)  # (2, P, L, N)
        joint = lp_cn + lp_rep + lp_reads
        terms["enum"] = torch.logsumexp(joint.reshape(2 * P, L, N), dim=0).sum()
    return terms


def elbo(prob: OracleProblem, z: Dict[str, torch.Tensor], **kw) -> torch.Tensor:
    c = constrain(prob.kind, z)
    return sum(model_terms(prob, c, **kw).values())


def loss_and_grads(prob: OracleProblem, z: Dict[str, torch.Tensor]):
    """-ELBO and d(-ELBO)/dz for every unconstrained param (what SVI.step feeds Adam)."""
    zz = {k: v.detach().clone().requires_grad_(True) for k, v in z.items()}
    loss = -elbo(prob, zz)
    loss.backward()
    return loss.detach(), {k: v.grad.detach() for k, v in zz.items()}


# --------------------------------------------------------------------------- init
def init_params(prob: OracleProblem, seed: int = 0, method: str = "sampled") -> Dict[str, torch.Tensor]:
    """AutoDelta initial values (B.4), returned unconstrained.

    ``sampled``: each univariate site takes the median of 15 draws from its prior,
    evaluated in model order with earlier sites at their initial values
    (``init_to_median(num_samples=15)``), from a torch.Generator seeded with
    ``seed`` -- the same distribution of inits as Pyro, not the same RNG stream.
    ``median``: the analytic prior medians (the num_samples -> infinity limit).
    The Dirichlet site falls back to a feasible point: transform_to(simplex)(0) = 1/P.
    """
    kind = prob.kind
    x = prob.reads.double()
    L, N = x.shape
    P, K = prob.P, prob.K
    g = torch.Generator().manual_seed(seed)
    c = {}

    def med(dist, shape, analytic):
        if method == "median":
            return analytic.expand(shape).clone().double()
        return _median_of_samples(dist, shape, g)

    if kind != "step3":
        ga = Gamma(torch.tensor([2.], dtype=torch.float64), torch.tensor([0.2], dtype=torch.float64))
        c["expose_a"] = med(ga, (1,), torch.tensor([_gamma_median(2.0, 0.2)], dtype=torch.float64))
    if kind == "step1":
        c["expose_lambda"] = torch.tensor([1e-1], dtype=torch.float64)          # lambda_init (:557)
        nb = Normal(torch.tensor(0., dtype=torch.float64), torch.tensor(1., dtype=torch.float64))
        c["expose_beta_means"] = med(nb, (prob.n_libs, K + 1), torch.tensor(0., dtype=torch.float64))
    c["expose_beta_stds"] = torch.logspace(start=0, end=-K, steps=K + 1, dtype=torch.float64
                                           ).reshape(1, -1).expand([prob.n_libs, K + 1]).clone()
    if kind != "step3":
        rb = Beta(torch.tensor([1.], dtype=torch.float64), torch.tensor([1.], dtype=torch.float64))
        c["expose_rho"] = med(rb, (L, 1), torch.tensor(0.5, dtype=torch.float64))
    if kind == "step1":
        tb = Beta(torch.tensor([1.5], dtype=torch.float64), torch.tensor([1.5], dtype=torch.float64))
        c["expose_tau"] = med(tb, (N,), torch.tensor(0.5, dtype=torch.float64))
    else:
        c["expose_tau"] = prob.t_init.double().clone()
    tau = transform_to(constraints.unit_interval)(
        transform_to(constraints.unit_interval).inv(c["expose_tau"]))
    ploidy = cell_ploidies(prob.to(torch.float64))
    u_guess = torch.mean(x, dim=0) / ((1 + tau) * ploidy)
    c["expose_u"] = med(Normal(u_guess, u_guess / 10.), (N,), u_guess)
    bm = c["expose_beta_means"] if kind == "step1" else prob.beta_means.double()
    bs = c["expose_beta_stds"]
    c["expose_betas"] = med(Normal(bm[prob.libs], bs[prob.libs]), (N, K + 1), bm[prob.libs])
    c["expose_pi"] = torch.full((L, N, P), 1.0 / P, dtype=torch.float64)
    z = unconstrain(kind, c)
    return {k: v.to(prob.reads.dtype) for k, v in z.items()}


def _gamma_median(conc: float, rate: float) -> float:
    from scipy.special import gammaincinv
    return float(gammaincinv(conc, 0.5) / rate)


def _median_of_samples(dist, shape, g: torch.Generator) -> torch.Tensor:
    """Median of 15 iid draws per element, drawn by inverse-CDF from ``g``."""
    shape = tuple(shape)
    batch = torch.broadcast_shapes(dist.batch_shape, shape) if len(dist.batch_shape) else shape
    uni = torch.rand((15,) + tuple(batch), generator=g, dtype=torch.float64).clamp(1e-12, 1 - 1e-12)
    if isinstance(dist, Normal):
        s = dist.loc + dist.scale * math.sqrt(2.0) * torch.erfinv(2 * uni - 1)
    elif isinstance(dist, (Gamma, Beta)):
        from scipy import stats
        if isinstance(dist, Gamma):
            s = torch.from_numpy(stats.gamma.ppf(uni.numpy(), a=dist.concentration.numpy(),
                                                 scale=1.0 / dist.rate.numpy()))
        else:
            s = torch.from_numpy(stats.beta.ppf(uni.numpy(), dist.concentration1.numpy(),
                                                dist.concentration0.numpy()))
    else:  # pragma: no cover
        raise TypeError(type(dist))
    return s.median(dim=0)[0].reshape(shape)


# --------------------------------------------------------------------------- SVI
@dataclass
class FitResult:
    z: Dict[str, torch.Tensor]
    losses: List[float] = field(default_factory=list)
    converged_at: Optional[int] = None
    nan_at: Optional[int] = None


def converged(losses: List[float], i: int, min_iter: int, rel_tol: float) -> bool:
    """pert_model.py:749-753 (also :807-811, :874-878)."""
    if i >= min_iter:
        loss_diff = abs(max(losses[-10:-1]) - min(losses[-10:-1])) / abs(losses[0] - losses[-1])
        return loss_diff < rel_tol
    return False


def fit(prob: OracleProblem, z0: Dict[str, torch.Tensor], lr: float = 0.05, max_iter: int = 100,
        min_iter: int = 10, rel_tol: float = 1e-6, cell_chunk: Optional[int] = None,
        callback=None) -> FitResult:
    """SVI loop of pert_model.py:742-758 / :800-816 / :867-883 with torch.optim.Adam."""
    params = {k: v.detach().clone().requires_grad_(True) for k, v in z0.items()}
    opt = torch.optim.Adam(list(params.values()), lr=lr, betas=ADAM_BETAS, eps=ADAM_EPS)
    res = FitResult(z=params)
    ploidy = cell_ploidies(prob)
    for i in range(max_iter):
        if cell_chunk is None:
            loss = -elbo(prob, params)
            loss.backward()
            lval = float(loss.detach())
        else:
            lval = _chunked_backward(prob, params, cell_chunk, ploidy)
        opt.step()
        opt.zero_grad()
        res.losses.append(lval)
        if callback is not None:
            callback(i, lval)
        if converged(res.losses, i, min_iter, rel_tol):
            res.converged_at = i
            break
        if np.isnan(lval):
            res.nan_at = i
            break
    res.z = {k: v.detach() for k, v in params.items()}
    return res


def _chunked_backward(prob: OracleProblem, params, cell_chunk: int, ploidy) -> float:
    """Gradient accumulation over cell chunks (mathematically identical to one pass)."""
    L, N = prob.reads.shape
    total = 0.0
    kind = prob.kind
    for j, s in enumerate(range(0, N, cell_chunk)):
        sl = slice(s, min(N, s + cell_chunk))
        sub = prob.cells(sl)
        zc = {}
        for name, _ in PARAM_SITES[kind]:
            v = params[name]
            if name in ("expose_tau", "expose_u", "expose_betas"):
                v = v[sl]
            elif name == "expose_pi":
                v = v[:, sl]
            zc[name] = v
        c = constrain(kind, zc)
        terms = model_terms(sub, c, global_terms=(j == 0), ploidy=ploidy[sl])
        loss = -sum(terms.values())
        loss.backward()
        total += float(loss.detach())
    return total


# --------------------------------------------------------------------------- decode
def enum_score_terms(prob: OracleProblem, z: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    """The (2, P, L, N) joint log score of (rep, cn) at the point z (steps 2/3) and its
    parts: ``lp_cn`` (P, L, N), ``lp_rep`` (2, 1, L, N), ``lp_reads`` (2, P, L, N), the
    parameter-free part of the reads term ``kappa`` (L, N: x log lam + x log x - x -
    lgamma(1 + x), the same for every state), ``delta`` and ``dpsi`` = d lp_reads / d delta
    (2, P, L, N; 0 where delta is clamped) -- the magnitudes an fp32 evaluation's rounding
    scales with (tests/_bounds.decode_mismatches)."""
    c = constrain(prob.kind, z)
    x = prob.reads
    L, N = x.shape
    P, K = prob.P, prob.K
    dt = x.dtype
    a = c["expose_a"] if prob.kind != "step3" else prob.a_fixed
    rho = c["expose_rho"] if prob.kind != "step3" else prob.rho_fixed
    tau, u, betas, pi = c["expose_tau"], c["expose_u"], c["expose_betas"], c["expose_pi"]
    lamb = prob.lamb
    t_diff = tau.reshape(-1, N) - rho.reshape(L, -1)
    phi = 1 / (1 + torch.exp(-a * t_diff))
    phi = torch.where(phi < 0.001, torch.full_like(phi, 0.001), phi)
    phi = torch.where(phi > 0.999, torch.full_like(phi, 0.999), phi)
    gcf = gc_features(prob.gc, K).reshape(L, 1, K + 1)
    omega = torch.exp(torch.sum(torch.mul(betas, gcf), 2))
    cn = torch.arange(P).reshape(P, 1, 1)
    rep = torch.tensor([0., 1.], dtype=dt).reshape(2, 1, 1, 1)
    chi = cn * (1. + rep)
    delta = u * chi * omega * (1 - lamb) / lamb
    clamped = delta < 1
    delta = torch.where(clamped, torch.ones_like(delta), delta)
    lp_cn = Categorical(pi).log_prob(cn)
    lp_rep = Bernoulli(phi).log_prob(rep)
    lp_reads = NegativeBinomial(delta, probs=lamb).log_prob(x)
    xlx = torch.where(x > 0, x * torch.log(torch.where(x > 0, x, torch.ones_like(x))), torch.zeros_like(x))
    kappa = x * torch.log(lamb) + xlx - x - torch.lgamma(1 + x)
    dpsi = torch.where(clamped, torch.zeros_like(delta),
                       torch.log1p(-lamb) + torch.digamma(delta + x) - torch.digamma(delta))
    return dict(score=lp_cn + lp_rep + lp_reads, lp_cn=lp_cn, lp_rep=lp_rep, lp_reads=lp_reads, kappa=kappa,
                delta=delta, dpsi=dpsi)


def enum_scores(prob: OracleProblem, z: Dict[str, torch.Tensor]) -> torch.Tensor:
    """(2, P, L, N) joint log score of (rep, cn) at the point z (steps 2/3)."""
    return enum_score_terms(prob, z)["score"]


@torch.no_grad()
def decode(prob: OracleProblem, z: Dict[str, torch.Tensor]):
    """infer_discrete(temperature=0) (pert_model.py:820-827, B.7): joint argmax.

    Returns cn (L, N) int64 and rep (L, N) float; ties resolve to the first
    state in (rep, cn) row-major order.
    """
    s = enum_scores(prob, z)
    P = prob.P
    L, N = prob.reads.shape
    idx = torch.argmax(s.reshape(2 * P, L, N), dim=0)
    return idx % P, (idx // P).to(prob.reads.dtype)


# --------------------------------------------------------------------------- constants
def dirichlet_normaliser_fp32(etas: torch.Tensor) -> float:
    """Sum over (bin, cell) of lgamma(sum eta) - sum lgamma(eta) evaluated with
    torch-CPU fp32 semantics (torch/distributions/dirichlet.py:93-97), accumulated
    in fp64 -- the parameter-free constant the reference adds to every loss."""
    e = etas.to(torch.float32)
    per = torch.lgamma(e.sum(-1)) - torch.lgamma(e).sum(-1)
    return float(per.double().sum())
