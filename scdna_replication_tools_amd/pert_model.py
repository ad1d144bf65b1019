"""Drop-in ``pert_infer_scRT`` (reference scdna_replication_tools/pert_model.py:36-901).

Same constructor arguments and defaults (:37-43), same ``run_pert_model()`` return
tuple ``(cn_s_out, supp_s_out_df, cn_g1_out, supp_g1_out_df)`` (:901) and output
columns (``model_cn_state``, ``model_rep_state``, ``model_tau``, ``model_u``,
``model_rho``; supp rows ``model_lambda``, ``model_a``, ``loss_g``, ``loss_s``,
:466-538).  The three SVI fits run on the GPU through libpert_hip.so
(``engine.PertShard``); there is no CPU path.

Extra keyword arguments (all optional): ``device`` (default ``cuda``),
``init_method`` ('sampled' = init_to_median(15) draws, 'median' = analytic medians),
``dirichlet_mode`` ('torch32' reproduces the reference's fp32 Dirichlet normaliser
in the reported losses, 'exact' = fp64), ``tau_init_method`` ('batched' = all cells'
GMM / threshold scan at once on the device, tau_init.py; 'sklearn' = the per-cell
sklearn loop) and ``n_jobs`` for the latter.
"""
from __future__ import annotations

import logging
import math
import time
from typing import List, Optional

import numpy as np
import pandas as pd
import torch

from . import prep
from ._native import KIND_STEP1, KIND_STEP2, KIND_STEP3
from .engine import EtaCodebook, PertShard
from .init import init_params
from .tau_init import guess_times_batched

log = logging.getLogger("scdna_replication_tools_amd.pert_model")


def _converged(losses: List[float], i: int, min_iter: int, rel_tol: float) -> bool:
    """pert_model.py:749-753 (also :807-811, :874-878)."""
    if i >= min_iter:
        loss_diff = abs(max(losses[-10:-1]) - min(losses[-10:-1])) / abs(losses[0] - losses[-1])
        return loss_diff < rel_tol
    return False


class pert_infer_scRT():
    def __init__(self, cn_s, cn_g1, input_col='reads', gc_col='gc', rt_prior_col='mcf7rt',
                 clone_col='clone_id', cell_col='cell_id', library_col='library_id',
                 chr_col='chr', start_col='start', cn_state_col='state', assign_col='copy',
                 rs_col='rt_state', frac_rt_col='frac_rt', cn_prior_method='g1_composite',
                 cn_prior_weight=1e6, learning_rate=0.05, max_iter=2000, min_iter=100, rel_tol=1e-6,
                 max_iter_step1=None, min_iter_step1=None, max_iter_step3=None, min_iter_step3=None,
                 cuda=False, seed=0, P=13, K=4, J=5, upsilon=6, run_step3=True, *, device=None,
                 init_method='sampled', dirichlet_mode='torch32', n_jobs=1, tau_init_method='batched'):
        self.cn_s = cn_s
        self.cn_g1 = cn_g1
        self.input_col = input_col
        self.gc_col = gc_col
        self.rt_prior_col = rt_prior_col
        self.clone_col = clone_col
        self.cell_col = cell_col
        self.library_col = library_col
        self.chr_col = chr_col
        self.start_col = start_col
        self.cn_state_col = cn_state_col
        self.assign_col = assign_col
        self.rs_col = rs_col
        self.frac_rt_col = frac_rt_col
        self.cn_prior_weight = cn_prior_weight
        self.learning_rate = learning_rate
        self.max_iter = max_iter
        self.min_iter = min_iter
        self.rel_tol = rel_tol
        self.cuda = cuda                      # accepted for compatibility; the fit always runs on the GPU
        self.seed = seed
        # step 1 / 3 default to half of step 2's limits (:104-120)
        self.max_iter_step1 = int(self.max_iter / 2) if max_iter_step1 is None else max_iter_step1
        self.min_iter_step1 = int(self.min_iter / 2) if min_iter_step1 is None else min_iter_step1
        self.max_iter_step3 = int(self.max_iter / 2) if max_iter_step3 is None else max_iter_step3
        self.min_iter_step3 = int(self.min_iter / 2) if min_iter_step3 is None else min_iter_step3
        self.cn_prior_method = cn_prior_method
        self.P = P
        self.L = None
        self.K = K
        self.J = J
        self.upsilon = upsilon
        self.run_step3 = run_step3
        self.device = torch.device(device) if device is not None else torch.device("cuda")
        self.init_method = init_method
        self.dirichlet_mode = dirichlet_mode
        self.n_jobs = n_jobs
        self.tau_init_method = tau_init_method
        self.timings = {}
        self.iters = {}

    # ------------------------------------------------------------------ prep
    def process_input_data(self):
        """pert_model.py:133-191 (vectorised, prep.process_input_data)."""
        self.cn_s, self.cn_g1, inp = prep.process_input_data(
            self.cn_s, self.cn_g1, input_col=self.input_col, gc_col=self.gc_col, cell_col=self.cell_col,
            library_col=self.library_col, chr_col=self.chr_col, start_col=self.start_col,
            cn_state_col=self.cn_state_col)
        self.L = len(inp.library_ids)
        return inp

    def build_etas(self, inp, profiles) -> EtaCodebook:
        """pert_model.py:668-716."""
        m, P, w = self.cn_prior_method, self.P, self.cn_prior_weight
        L, N = inp.reads_s.shape
        if m == 'hmmcopy':
            return prep.build_cn_prior(inp.states_s, w, P)
        if m == 'g1_cells':
            return prep.build_g1_cells_prior(inp, self.cn_s, self.cn_g1, w, P, self.cell_col, self.clone_col)
        if m == 'g1_clones':
            return prep.build_clone_cn_prior(self.cn_s, inp.cells_s, inp.loci_chr, inp.loci_start, profiles, w, P,
                                             self.cell_col, self.clone_col, keys=inp.keys_s)
        if m == 'g1_composite':
            return prep.build_composite_cn_prior(inp, self.cn_s, self.cn_g1, profiles, P, J=self.J,
                                                 cell_col=self.cell_col, clone_col=self.clone_col,
                                                 cn_state_col=self.cn_state_col)
        if m == 'diploid':
            return prep.diploid_prior(L, N, w, P)
        return prep.uniform_prior(L, N, P)

    def guess_times(self, reads, cn_states):
        """pert_model.py:426-457: (t_init, t_alpha_prior, t_beta_prior)."""
        if self.tau_init_method == 'sklearn':
            return prep.guess_times(reads, cn_states, self.upsilon, self.n_jobs)
        return guess_times_batched(reads, cn_states, self.upsilon, device=self.device)

    # ------------------------------------------------------------------ fits
    def _svi(self, shard: PertShard, max_iter: int, min_iter: int, label: str) -> List[float]:
        """The SVI loop of pert_model.py:742-758 (also :800-816, :867-883).  The loss
        record and the stopping rule run on the device (PertShard.run_svi), so the host
        queues iterations without a per-step synchronisation; the losses, log lines and
        stopping iteration are the ones the host loop below would produce:

            for i in range(max_iter):
                losses.append(svi.step(...))
                if i >= min_iter and plateau(losses) < rel_tol: break
                if isnan(losses[-1]): break
        """
        t0 = time.perf_counter()
        losses, reason = shard.run_svi(max_iter, min_iter, self.rel_tol)
        for i, loss in enumerate(losses):
            log.info('step: {}, loss: {}'.format(i, loss))
        if reason == 1:
            print('ELBO converged at iteration ' + str(len(losses) - 1))
        elif reason == 2:
            print('ELBO is NaN at iteration ' + str(len(losses) - 1))
        self.timings[label] = time.perf_counter() - t0
        self.iters[label] = len(losses)
        return losses

    def run_pert_model(self):
        t_all = time.perf_counter()
        P, K = self.P, self.K
        tic = time.perf_counter()
        inp = self.process_input_data()
        n_libs = self.L
        profiles = prep.consensus_clone_profiles(
            self.cn_g1, self.cn_state_col, clone_col=self.clone_col, cell_col=self.cell_col,
            chr_col=self.chr_col, start_col=self.start_col, cn_state_col=self.cn_state_col, keys=inp.keys_g)
        etas = self.build_etas(inp, profiles)
        self.timings["prep"] = time.perf_counter() - tic

        # ---- step 1: G1/2 cells doubled, cn / rep observed (:718-774)
        st_g2, rd_g2, lb_g2, rep_g2 = prep.make_g1_g2_training_data(inp.states_g, inp.reads_g, inp.libs_g)
        init1 = init_params(KIND_STEP1, rd_g2, lb_g2, n_libs, P, K, seed=self.seed, method=self.init_method)
        s1 = PertShard(KIND_STEP1, rd_g2, inp.gc, lb_g2, n_libs, P, K, init1, cn_obs=st_g2, rep_obs=rep_g2,
                       device=self.device, lr=self.learning_rate, dirichlet_mode=self.dirichlet_mode)
        logging.info('STEP 1: Learning reads to CN bias from low variance cells.')
        losses_g = self._svi(s1, self.max_iter_step1, self.min_iter_step1, "step1")
        c1 = s1.constrained()
        lambda_fit = np.asarray(c1["expose_lambda"], dtype=np.float32)
        beta_means_fit = np.asarray(c1["expose_beta_means"], dtype=np.float32)
        del s1

        # ---- step 2: S cells, enumerated (:776-830)
        tic = time.perf_counter()
        t_init, _, _ = self.guess_times(inp.reads_s, etas.argmax_states())
        self.timings["guess_times_s"] = time.perf_counter() - tic
        ploidy = etas.argmax_states().astype(np.float32).mean(0)
        init2 = init_params(KIND_STEP2, inp.reads_s, inp.libs_s, n_libs, P, K, ploidy=ploidy, t_init=t_init,
                            beta_means=beta_means_fit, seed=self.seed, method=self.init_method)
        s2 = PertShard(KIND_STEP2, inp.reads_s, inp.gc, inp.libs_s, n_libs, P, K, init2, eta=etas,
                       lamb=float(lambda_fit[0]), beta_means=beta_means_fit, device=self.device,
                       lr=self.learning_rate, dirichlet_mode=self.dirichlet_mode)
        logging.info('STEP 2: Jointly infer replication and CN states in high variance cells.')
        losses_s = self._svi(s2, self.max_iter, self.min_iter, "step2")
        tic = time.perf_counter()
        cn_map, rep_map = s2.decode()
        c2 = s2.constrained()
        cn_s_out, supp_s_out_df = self.package_s_output(
            self.cn_s, inp.cells_s, inp.loci_chr, inp.loci_start, cn_map.cpu().numpy(), rep_map.cpu().numpy(),
            c2, lambda_fit, losses_g, losses_s, keys=inp.keys_s)
        self.timings["decode_package_s"] = time.perf_counter() - tic
        rho_fit = c2["expose_rho"]
        a_fit = c2["expose_a"]
        del s2

        cn_g1_out = supp_g1_out_df = None
        if self.run_step3:
            # ---- step 3: G1 cells with rho, a frozen (:834-896)
            tic = time.perf_counter()
            etas2 = prep.build_clone_cn_prior(self.cn_g1, inp.cells_g, inp.loci_chr, inp.loci_start, profiles,
                                              self.cn_prior_weight, P, self.cell_col, self.clone_col, keys=inp.keys_g)
            t_init2, _, _ = self.guess_times(inp.reads_g, etas2.argmax_states())
            ploidy2 = etas2.argmax_states().astype(np.float32).mean(0)
            self.timings["prep_step3"] = time.perf_counter() - tic
            init3 = init_params(KIND_STEP3, inp.reads_g, inp.libs_g, n_libs, P, K, ploidy=ploidy2,
                                t_init=t_init2, beta_means=beta_means_fit, seed=self.seed, method=self.init_method)
            s3 = PertShard(KIND_STEP3, inp.reads_g, inp.gc, inp.libs_g, n_libs, P, K, init3, eta=etas2,
                           lamb=float(lambda_fit[0]), beta_means=beta_means_fit,
                           rho_fixed=np.asarray(rho_fit).reshape(-1), a_fixed=float(np.asarray(a_fit)[0]),
                           device=self.device, lr=self.learning_rate, dirichlet_mode=self.dirichlet_mode)
            logging.info('STEP 3: Running pre-trained S-phase model on low variance cells.')
            losses_s2 = self._svi(s3, self.max_iter_step3, self.min_iter_step3, "step3")
            tic = time.perf_counter()
            cn3, rep3 = s3.decode()
            c3 = s3.constrained()
            c3["expose_rho"] = rho_fit
            c3["expose_a"] = a_fit
            cn_g1_out, supp_g1_out_df = self.package_s_output(
                self.cn_g1, inp.cells_g, inp.loci_chr, inp.loci_start, cn3.cpu().numpy(), rep3.cpu().numpy(),
                c3, lambda_fit, losses_g, losses_s2, keys=inp.keys_g)
            self.timings["decode_package_g"] = time.perf_counter() - tic
            del s3
        self.timings["total"] = time.perf_counter() - t_all
        return cn_s_out, supp_s_out_df, cn_g1_out, supp_g1_out_df

    # ------------------------------------------------------------------ outputs
    def package_s_output(self, cn, cells, loci_chr, loci_start, model_cn, model_rep, fit, lambda_fit,
                         losses_g, losses_s, keys=None):
        """pert_model.py:466-538: per (bin, cell) model_cn_state / model_rep_state, per cell
        model_tau / model_u, per bin model_rho (inner joins on the long table), plus the
        supp frame of lambda, a and the loss traces."""
        if keys is not None and len(keys.cell_code) == len(cn):
            ci, li = keys.row_positions(cells, loci_chr, loci_start)
        else:
            cell_index = pd.Index(np.asarray(cells).astype(str))
            locus_index = pd.MultiIndex.from_arrays([np.asarray(loci_chr).astype(str), np.asarray(loci_start)])
            ci = cell_index.get_indexer(cn[self.cell_col].astype(str).to_numpy())
            li = locus_index.get_indexer(pd.MultiIndex.from_arrays(
                [cn[self.chr_col].astype(str).to_numpy(), cn[self.start_col].to_numpy()]))
        keep = (ci >= 0) & (li >= 0)
        base = cn.loc[keep] if not keep.all() else cn
        ci, li = ci[keep], li[keep]
        model = pd.DataFrame({
            'model_cn_state': model_cn[li, ci].astype(np.int64),
            'model_rep_state': model_rep[li, ci].astype(np.float32),
            'model_tau': np.asarray(fit["expose_tau"], dtype=np.float32)[ci],
            'model_u': np.asarray(fit["expose_u"], dtype=np.float32)[ci],
            'model_rho': np.asarray(fit["expose_rho"], dtype=np.float32).reshape(-1)[li],
        })
        # new columns side by side with the (sorted) input rows, without copying its blocks
        # (reset_index(drop=True) would deep-copy and consolidate the whole long table)
        base = base.copy(deep=False)
        base.index = pd.RangeIndex(len(base))
        out = pd.concat([base, model], axis=1, copy=False)
        supp = pd.concat([
            pd.DataFrame({'param': ['model_lambda'], 'level': ['all'], 'value': [float(lambda_fit[0])]}),
            pd.DataFrame({'param': ['model_a'], 'level': ['all'], 'value': [float(np.asarray(fit["expose_a"])[0])]}),
            pd.DataFrame({'param': ['loss_g'] * len(losses_g), 'level': np.arange(len(losses_g)), 'value': losses_g}),
            pd.DataFrame({'param': ['loss_s'] * len(losses_s), 'level': np.arange(len(losses_s)), 'value': losses_s}),
        ], ignore_index=True)
        return out, supp
