"""Where does step 2's stopping iteration come from?  (test infrastructure, CPU only)

Re-runs step 2 of the genome-length oracle chain (tests/golden/make_genome_chain_golden.py)
alone, from the fixture's step-1 sites (lambda, beta_means) and t_init, in variants of the
per-element arithmetic, and prints where pert_model.py:807-811's rule stops each one:

  ref          the fp32 oracle as committed (torch autograd of torch.distributions, the
               tensor algebra Pyro runs) -- must reproduce the fixture's trace and stop
  logsoftmax   the Dirichlet term's xlogy(eta-1, pi) evaluated as (eta-1) * log_softmax(z):
               the same value, but its gradient is cancellation-free (the product's form,
               SURVEY.md Appendix C) instead of (eta-1)/pi pushed back through the softmax
  detach_max   SoftmaxTransform with its max detached (mathematically the same gradient;
               in fp32 the softmax backward's residue sum_k dL/dp_k p_k no longer lands on
               the argmax logit)
  exp64        SoftmaxTransform's exponential correctly rounded (through fp64): the same
               fp32 autograd structure with other last bits in pi
  product      the reference's forward values with the product kernel's pi-logit gradient
               pi_k (S1 + sum gcm) - W_k - gcm_k (clamp masks in log space); "_domfix": the
               argmax logit's gradient as minus the others' sum (the reference's max path),
               "_refmask": the clamp masks of clamp_probs(pi / sum pi) in fp32

Results (profiles/r04_stop_probe.log): ref at 4 threads and under ATEN_CPU_CAPABILITY=avx2
stop at 1,151 like the fixture; detach_max at 1,151; logsoftmax -- whose gradient quantises
W (1 - pi_argmax) like the product's per-element form once fp32 pi_argmax rounds to 1 -- at
1,178, where the product stopped; product_domfix (and _refmask) at 1,151.

Run under ``ATEN_CPU_CAPABILITY=default|avx2|avx512`` for the reference's own fp32 arithmetic
on CPUs with other vector units (torch CPU picks its exp / log / reduction kernels by ISA).

    python tools/stop_probe.py ref [--threads 4] [--out file.npz]
"""
import argparse
import math
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import pert_oracle as po  # noqa: E402
from tests._chain import _t, _z0  # noqa: E402
from tests._configs import genome_scrt, genome_tables  # noqa: E402
from scdna_replication_tools_amd import prep  # noqa: E402
from scdna_replication_tools_amd.init import init_params  # noqa: E402

FIXTURE = os.path.join(ROOT, "tests", "golden", "genome_chain_oracle.npz")


def _patch(variant):
    if variant == "detach_max":
        from torch.distributions.transforms import SoftmaxTransform

        def _call(self, x):
            probs = (x - x.max(-1, True)[0].detach()).exp()
            return probs / probs.sum(-1, True)
        SoftmaxTransform._call = _call
    elif variant == "exp64":
        from torch.distributions.transforms import SoftmaxTransform

        def _call(self, x):
            probs = (x - x.max(-1, True)[0]).double().exp().float()   # correctly rounded exp
            return probs / probs.sum(-1, True)
        SoftmaxTransform._call = _call
    elif variant.startswith("product"):
        # the pi site's forward values as the reference computes them, its gradient as the
        # product's kernel forms it: d(-ELBO)/dz_k = pi_k (S1 + sum_j gcm_j) - W_k - gcm_k with
        # gcm_k = gamma_k * mask_k; "_domfix": the argmax logit's gradient as minus the sum of
        # the others (what the reference's max path gives); "_refmask": the clamp masks of
        # clamp_probs(pi / sum pi) in fp32 (the reference's), not in log space
        domfix = "domfix" in variant
        refmask = "refmask" in variant
        eps = float(torch.finfo(torch.float32).eps)

        class PiSite(torch.autograd.Function):
            @staticmethod
            def forward(ctx, z, W):
                mx = z.max(-1, True)[0]
                p = (z - mx).exp()
                pi = p / p.sum(-1, True)
                pi2 = pi / pi.sum(-1, keepdim=True)
                lc = torch.log(pi2.clamp(min=eps, max=1 - eps))
                dirv = torch.xlogy(W, pi).sum(-1)
                if refmask:
                    mask = (pi2 >= eps) & (pi2 <= 1 - eps)
                else:
                    lz = torch.log_softmax(z, -1)
                    mask = (lz >= math.log(eps)) & (lz <= math.log1p(-eps))
                ctx.save_for_backward(z, W, mask)
                return dirv, lc

            @staticmethod
            def backward(ctx, g_dir, g_lc):
                z, W, mask = ctx.saved_tensors
                gcm = torch.where(mask, -g_lc, torch.zeros_like(g_lc))          # gamma_k [unclamped]
                pk = torch.softmax(z, -1)
                S1 = W.sum(-1, keepdim=True)
                gl = pk * (S1 + gcm.sum(-1, keepdim=True)) - W - gcm               # d(-ELBO)/dz
                if domfix:
                    jm = z.argmax(-1, keepdim=True)
                    others = gl.scatter(-1, jm, torch.zeros_like(jm, dtype=gl.dtype)).sum(-1, keepdim=True)
                    gl = gl.scatter(-1, jm, -others)
                return gl * (-g_dir).unsqueeze(-1), None

        def elbo(prob, z, **kw):
            c = po.constrain(prob.kind, z)
            e = prob.etas
            dirv, lc = PiSite.apply(z["expose_pi"], e - 1.0)
            orig_dir, orig_cat = po.Dirichlet, po.Categorical

            class _Dir:                                   # Dirichlet(etas).log_prob(pi) -> site value
                def __init__(self, conc):
                    self.conc = conc

                def log_prob(self, value):
                    return dirv + torch.lgamma(self.conc.sum(-1)) - torch.lgamma(self.conc).sum(-1)

            class _Cat:                                   # Categorical(pi).log_prob(cn) -> lc permuted
                def __init__(self, probs):
                    pass

                def log_prob(self, value):
                    return lc.permute(2, 0, 1)
            po.Dirichlet, po.Categorical = _Dir, _Cat
            try:
                terms = po.model_terms(prob, c, **kw)
            finally:
                po.Dirichlet, po.Categorical = orig_dir, orig_cat
            return sum(terms.values())
        po.elbo = elbo
    elif variant == "logsoftmax":
        base = po.elbo

        def elbo(prob, z, **kw):
            c = po.constrain(prob.kind, z)
            terms = po.model_terms(prob, c, **kw)
            e = prob.etas
            terms["expose_pi"] = ((e - 1.0) * torch.log_softmax(z["expose_pi"], -1)).sum() + (
                torch.lgamma(e.sum(-1)) - torch.lgamma(e).sum(-1)).sum()
            return sum(terms.values())
        po.elbo = elbo
        assert base is not po.elbo
    elif variant == "contdir":
        # the reference's arithmetic for the gradient, but the Dirichlet site's VALUE in the
        # loss record without the reference's per-element fp32 rounding: (eta - 1) log pi summed
        # and the normaliser added in fp64 (what a kernel with an fp64 accumulator records)
        base = po.elbo

        def elbo(prob, z, **kw):
            c = po.constrain(prob.kind, z)
            terms = po.model_terms(prob, c, **kw)
            e = prob.etas.double()
            zp = z["expose_pi"].double()
            cont = ((e - 1.0) * torch.log_softmax(zp, -1)).sum() + (torch.lgamma(e.sum(-1)) - torch.lgamma(e).sum(-1)).sum()
            ref = terms["expose_pi"]
            total = sum(terms.values())
            return total + (cont - ref.double()).detach().to(total.dtype)
        po.elbo = elbo
        assert base is not po.elbo
    elif variant != "ref":
        raise SystemExit("unknown variant " + variant)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variant")
    ap.add_argument("--threads", type=int, default=4)
    ap.add_argument("--max-iter", type=int, default=None)
    ap.add_argument("--out", default=None)
    ap.add_argument("--step1-from", default=None,
                    help="an .npz holding lam (and beta_means): start step 2 from those step-1 sites "
                         "instead of the fixture's (e.g. the product's dump of the same chain)")
    a = ap.parse_args()
    torch.set_num_threads(a.threads)
    _patch(a.variant)
    fx = dict(np.load(FIXTURE))
    s, g, _ = genome_tables()
    m = genome_scrt(s, g, device="cpu")._pert_model()
    inp = m._prepare()
    P, K, nl = m.P, m.K, m.L
    profiles = prep.consensus_clone_profiles(m.cn_g1, m.cn_state_col, clone_col=m.clone_col, cell_col=m.cell_col,
                                             chr_col=m.chr_col, start_col=m.start_col, cn_state_col=m.cn_state_col,
                                             keys=inp.keys_g)
    etas = m._build_etas(inp, profiles)
    lam, bm, t_init = fx["lam"], fx["beta_means"], fx["t_init_s"]
    if a.step1_from:
        alt = dict(np.load(a.step1_from))
        lam = np.asarray(alt["lam"], np.float32).reshape(np.shape(lam))
        if "beta_means" in alt:
            bm = np.asarray(alt["beta_means"], np.float32).reshape(np.shape(bm))
    dt = torch.float32
    ploidy = etas.argmax_states().astype(np.float32).mean(0)
    L, N = inp.reads_s.shape
    init2 = init_params(2, inp.reads_s, inp.libs_s, nl, P, K, ploidy=ploidy, t_init=t_init, beta_means=bm,
                        seed=m.seed, method=m.init_method)
    prob = po.OracleProblem("step2", _t(inp.reads_s, dt), _t(inp.gc, dt), torch.as_tensor(inp.libs_s, dtype=torch.long),
                            nl, P, K, etas=_t(etas.dense(), dt), lamb=_t(lam, dt), beta_means=_t(bm, dt),
                            t_init=_t(t_init, dt))
    t0 = time.perf_counter()

    def cb(i, lval):
        if i % 50 == 0:
            ref = fx["losses_s"][i] if i < len(fx["losses_s"]) else float("nan")
            print("it {} loss {:.1f} fixture {:.1f} {:.0f}s".format(i, lval, ref, time.perf_counter() - t0), flush=True)
    r = po.fit(prob, _z0("step2", init2, L, N, P, dt), lr=m.learning_rate, max_iter=a.max_iter or m.max_iter,
               min_iter=m.min_iter, rel_tol=m.rel_tol, callback=cb)
    losses = np.asarray(r.losses)
    n = min(len(losses), len(fx["losses_s"]))
    dev = np.abs(losses[:n] - fx["losses_s"][:n])
    cap = torch.backends.cpu.get_cpu_capability()
    print("variant {} capability {} stop {} (fixture {}) first-iteration dev {:.1f} max dev {:.1f} at {}".format(
        a.variant, cap, len(losses), len(fx["losses_s"]), dev[0], dev.max(), int(dev.argmax())), flush=True)
    if a.out:
        np.savez_compressed(a.out, losses=losses, variant=a.variant, capability=cap)


if __name__ == "__main__":
    main()
