"""Drop-in ``pert_infer_scRT`` (reference scdna_replication_tools/pert_model.py:36-901).

Same constructor arguments and defaults (:37-43), same ``run_pert_model()`` return
tuple ``(cn_s_out, supp_s_out_df, cn_g1_out, supp_g1_out_df)`` (:901) and output
columns (``model_cn_state``, ``model_rep_state``, ``model_tau``, ``model_u``,
``model_rho``; supp rows ``model_lambda``, ``model_a``, ``loss_g``, ``loss_s``,
:466-538), and the reference's public helper methods with their signatures
(``process_input_data`` :133, ``sort_by_cell_and_loci`` :194, ``get_libraries_tensor``
:206, ``make_g1_g2_training_data`` :228, ``convert_rt_prior_units`` :254,
``build_trans_mat`` :260, ``build_cn_prior`` :272, ``build_clone_cn_prior`` :285,
``build_composite_cn_prior`` :299, ``manhattan_binarization`` :364, ``guess_times`` :426,
``make_gc_features`` :460, ``package_s_output`` :466).  ``model_s`` (:541, a Pyro model)
has no counterpart: the SVI fits run on the GPU through libpert_hip.so
(``engine.PertShard``); there is no CPU path.

Under ``torch.distributed`` (one process per GPU, world size > 1) every fit is
cell-sharded over the ranks with one all-reduce of the shared-gradient block per step
(sharding.py); every rank returns the full outputs.

Extra keyword arguments (all optional): ``device`` (default ``cuda``, or
``cuda:<LOCAL_RANK>`` under torch.distributed), ``init_method`` ('sampled' =
init_to_median(15) draws, 'median' = analytic medians), ``dirichlet_mode`` ('torch32'
reproduces the reference's fp32 Dirichlet normaliser in the reported losses, 'exact' =
fp64), ``tau_init_method`` ('batched' = all cells' GMM / threshold scan at once on the
device plus the exact host path for the cells rounding could change, tau_init.py;
'sklearn' = the per-cell sklearn loop), ``n_jobs`` (threads of either; no worker processes),
``process_group`` (a torch.distributed group; default: the world when initialised) and
``log_steps`` (False: no per-step 'step: i, loss: ...' log lines).
"""
from __future__ import annotations

import contextlib
import logging
import os
import time
from typing import List, Optional

import numpy as np
import pandas as pd
import torch

from . import prep
from ._native import KIND_STEP1, KIND_STEP2, KIND_STEP3
from .engine import CanonicalPiBlock, EtaCodebook, PertShard
from .init import init_params
from .sharding import cell_bounds, make_allreduce
from .tau_init import default_threads, guess_times_batched, host_threads

log = logging.getLogger("scdna_replication_tools_amd.pert_model")

_REF_LOGGING = []


def configure_reference_logging():
    """The logging set-up the reference runs when pert_model is imported
    (pert_model.py:25-33): root logger at DEBUG with basicConfig's stderr handler
    (format '%(relativeCreated) 9d %(message)s') plus a stdout handler for DEBUG records,
    so the per-step 'step: i, loss: ...' lines of every fit are visible.  Done once per
    process; the drop-in module ``scdna_replication_tools.pert_model`` calls it at import,
    as the reference does.  ``pert_infer_scRT(..., log_steps=False)`` silences the per-step
    lines of a fit."""
    if _REF_LOGGING:
        return
    import sys
    logging.basicConfig(format='%(relativeCreated) 9d %(message)s', level=logging.DEBUG)
    root = logging.getLogger()
    h = logging.StreamHandler(sys.stdout)
    h.setLevel(logging.DEBUG)
    h.addFilter(lambda record: record.levelno <= logging.DEBUG)
    root.addHandler(h)
    _REF_LOGGING.append(h)


def _converged(losses: List[float], i: int, min_iter: int, rel_tol: float) -> bool:
    """pert_model.py:749-753 (also :807-811, :874-878)."""
    if i >= min_iter:
        loss_diff = abs(max(losses[-10:-1]) - min(losses[-10:-1])) / abs(losses[0] - losses[-1])
        return loss_diff < rel_tol
    return False


def _np(v):
    if isinstance(v, torch.Tensor):
        return v.detach().cpu().numpy()
    return np.asarray(v)


class MapTrace:
    """The part of a Pyro trace that ``package_s_output`` reads (``trace.nodes[name]['value']``),
    for the MAP values of one fit: expose_u / expose_rho / expose_a / expose_tau and the
    decoded ``cn`` / ``rep`` (pert_model.py:472-477)."""

    def __init__(self, **values):
        self.nodes = {k: {"value": v} for k, v in values.items()}


class PivotAxes:
    """``index`` (loci: MultiIndex chr, start) and ``columns`` (cells) of the reference's
    (loci x cells) read-count frame -- all ``package_s_output`` uses of ``cn_s_reads_df``
    (:480-499) -- without materialising the frame; ``keys`` carries the sorted long table's
    integer keys for the fast row lookup."""

    def __init__(self, loci_chr, loci_start, cells, chr_col="chr", start_col="start", cell_col="cell_id",
                 keys=None):
        # chr as the category sort_by_cell_and_loci made it (:196-201), as pivot_table keeps it
        chr_lvl = pd.Categorical(np.asarray(loci_chr).astype(str), categories=prep.CHR_ORDER)
        self.index = pd.MultiIndex.from_arrays([chr_lvl, np.asarray(loci_start)], names=[chr_col, start_col])
        self.columns = pd.Index(np.asarray(cells), name=cell_col)
        self.keys = keys


class _Dist:
    """The process group a fit is sharded over (world 1 = no sharding)."""

    def __init__(self, group=None, device=None):
        import torch.distributed as dist
        self.dist = dist if dist.is_available() and dist.is_initialized() else None
        self.group = group
        self.world = self.dist.get_world_size(group) if self.dist else 1
        self.rank = self.dist.get_rank(group) if self.dist else 0
        self.backend = self.dist.get_backend(group) if self.dist else None
        # ranks on RCCL (one process per GPU): a pert_comm communicator of the library's own, so
        # each fit's SVI loop -- all-reduce included -- is one GIL-free C call; other backends
        # (gloo: several ranks sharing a GPU in tests) all-reduce through torch.distributed per
        # step, or -- PERT_NATIVE_COMM=host -- through the library's host-staged communicator
        # (the same C loop as RCCL ranks run).  The choice is collective: a communicator that
        # fails on any rank fails on all of them (engine.RcclComm), and all fall back together.
        self.comm = None
        mode = os.environ.get("PERT_NATIVE_COMM", "1")
        if self.world > 1 and mode == "host":
            from .engine import HostComm
            self.comm = HostComm(group)
        elif self.world > 1 and self.backend == "nccl" and mode != "0":
            from .engine import RcclComm
            try:
                self.comm = RcclComm(group, device=device)
            except Exception as e:                 # noqa: BLE001  (torch.distributed's all-reduce then)
                log.warning("the library's RCCL communicator failed (%s: %s); all-reducing through "
                            "torch.distributed per step", type(e).__name__, e)
        self.allreduce = (self.comm.allreduce if self.comm is not None else
                          make_allreduce(group) if self.world > 1 else None)

    def close(self):
        if self.comm is not None:
            self.comm.close()
            self.comm = None

    def bounds(self, n: int):
        return cell_bounds(n, self.world)[self.rank]

    def gather_cells(self, a: np.ndarray) -> np.ndarray:
        """Concatenate the ranks' cell-axis (last axis) blocks of ``a`` in rank order."""
        if self.world == 1:
            return a
        dev = torch.device("cuda", torch.cuda.current_device()) if self.backend == "nccl" else torch.device("cpu")
        t = torch.as_tensor(np.ascontiguousarray(a)).to(dev)
        n = torch.tensor([t.shape[-1]], device=dev)
        ns = [torch.zeros_like(n) for _ in range(self.world)]
        self.dist.all_gather(ns, n, group=self.group)
        ns = [int(x.item()) for x in ns]
        pad = torch.zeros(t.shape[:-1] + (max(ns),), dtype=t.dtype, device=dev)
        pad[..., :t.shape[-1]] = t
        parts = [torch.empty_like(pad) for _ in range(self.world)]
        self.dist.all_gather(parts, pad, group=self.group)
        return torch.cat([p[..., :k] for p, k in zip(parts, ns)], dim=-1).cpu().numpy()


class pert_infer_scRT():
    def __init__(self, cn_s, cn_g1, input_col='reads', gc_col='gc', rt_prior_col='mcf7rt',
                 clone_col='clone_id', cell_col='cell_id', library_col='library_id',
                 chr_col='chr', start_col='start', cn_state_col='state', assign_col='copy',
                 rs_col='rt_state', frac_rt_col='frac_rt', cn_prior_method='g1_composite',
                 cn_prior_weight=1e6, learning_rate=0.05, max_iter=2000, min_iter=100, rel_tol=1e-6,
                 max_iter_step1=None, min_iter_step1=None, max_iter_step3=None, min_iter_step3=None,
                 cuda=False, seed=0, P=13, K=4, J=5, upsilon=6, run_step3=True, *, device=None,
                 init_method='sampled', dirichlet_mode='torch32', n_jobs=1, tau_init_method='batched',
                 process_group=None, log_steps=True):
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
        self.L = None                         # number of libraries (:214)
        self.K = K
        self.J = J
        self.upsilon = upsilon
        self.run_step3 = run_step3
        self._group = process_group
        if device is None:
            dist = torch.distributed
            lr = int(os.environ.get("LOCAL_RANK", "0")) if dist.is_available() and dist.is_initialized() else None
            device = "cuda" if lr is None else "cuda:{}".format(lr)
        self.device = torch.device(device)
        self.init_method = init_method
        self.dirichlet_mode = dirichlet_mode
        self.n_jobs = n_jobs
        # threads of the tau initialiser's exact host path (no worker processes): one
        # (tau_init.default_threads) unless n_jobs > 1 names a count
        self.tau_threads = n_jobs if n_jobs > 1 else default_threads()
        self.tau_init_method = tau_init_method
        self.log_steps = log_steps
        self.timings = {}
        self.iters = {}
        self.launched = {}
        self._inp = None

    # the input tables: after _prepare, their sorted copies -- possibly still being built on a
    # background thread (prep.DeferredTable), in which case reading the attribute waits for it;
    # the priors take per-cell labels from the raw attribute without waiting (_raw_table)
    @property
    def cn_s(self):
        if isinstance(self._cn_s, prep.DeferredTable):
            self._cn_s = self._cn_s.result()
        return self._cn_s

    @cn_s.setter
    def cn_s(self, v):
        self._cn_s = v

    @property
    def cn_g1(self):
        if isinstance(self._cn_g1, prep.DeferredTable):
            self._cn_g1 = self._cn_g1.result()
        return self._cn_g1

    @cn_g1.setter
    def cn_g1(self, v):
        self._cn_g1 = v

    def _raw_table(self, which: str):
        return self._cn_s if which == "s" else self._cn_g1

    # ------------------------------------------------------------------ prep (host)
    def _prepare(self, on_g1_sorted=None, defer_sorted: bool = False) -> prep.PertInputs:
        """pert_model.py:133-191, vectorised (prep.process_input_data): sorts and filters
        self.cn_s / self.cn_g1 like the reference and returns the tensor inputs.
        ``defer_sorted``: the sorted copies of per-cell-block tables are built on a background
        thread (run_pert_model: the fit starts from the pivots; packaging takes the copies)."""
        if self._inp is None:
            self.cn_s, self.cn_g1, inp = prep.process_input_data(
                self._cn_s, self._cn_g1, input_col=self.input_col, gc_col=self.gc_col, cell_col=self.cell_col,
                library_col=self.library_col, chr_col=self.chr_col, start_col=self.start_col,
                cn_state_col=self.cn_state_col, on_g1_sorted=on_g1_sorted, defer_sorted=defer_sorted)
            self.L = len(inp.library_ids)
            self._inp = inp
        return self._inp

    def _long_rows(self) -> int:
        """Rows of the two input tables (cells x bins), before any preparation."""
        return int(len(self.cn_s)) + int(len(self.cn_g1))

    def _axes(self, cells, keys=None) -> PivotAxes:
        inp = self._prepare()
        return PivotAxes(inp.loci_chr, inp.loci_start, cells, self.chr_col, self.start_col, self.cell_col, keys)

    def _frame(self, values, cells) -> pd.DataFrame:
        ax = self._axes(cells)
        return pd.DataFrame(values, index=ax.index, columns=ax.columns)

    def process_input_data(self):
        """pert_model.py:133-191: returns the reference's 12-tuple (cn_g1_reads_df,
        cn_g1_states_df, cn_s_reads_df, cn_s_states_df, cn_g1_reads, cn_g1_states, cn_s_reads,
        cn_s_states, gammas, rt_prior_profile, libs_g1, libs_s).  The (loci x cells) frames
        hold the int64-truncated values the tensors hold."""
        inp = self._prepare()
        t = lambda a: torch.as_tensor(np.asarray(a, np.float32))
        rt_prior = None
        if self.rt_prior_col is not None and self.rt_prior_col in self.cn_s.columns:
            prof = self.cn_s[[self.chr_col, self.start_col, self.rt_prior_col]].drop_duplicates().dropna()
            rt_prior = self.convert_rt_prior_units(
                torch.tensor(prof[self.rt_prior_col].values).unsqueeze(-1).to(torch.float32))
        return (self._frame(inp.reads_g, inp.cells_g), self._frame(inp.states_g, inp.cells_g),
                self._frame(inp.reads_s, inp.cells_s), self._frame(inp.states_s, inp.cells_s),
                t(inp.reads_g), t(inp.states_g), t(inp.reads_s), t(inp.states_s), t(inp.gc), rt_prior,
                torch.as_tensor(inp.libs_g), torch.as_tensor(inp.libs_s))

    def sort_by_cell_and_loci(self, cn):
        """pert_model.py:194-203."""
        return prep.sort_by_cell_and_loci(cn, self.cell_col, self.chr_col, self.start_col)

    def get_libraries_tensor(self, cn_s, cn_g1):
        """pert_model.py:206-225: per-cell library index (first-appearance order over S then
        G1 cells), as int64 tensors; sets self.L to the number of libraries."""
        libs_s = cn_s[[self.cell_col, self.library_col]].drop_duplicates()
        libs_g1 = cn_g1[[self.cell_col, self.library_col]].drop_duplicates()
        ids = pd.concat([libs_s, libs_g1])[self.library_col].unique()
        self.L = int(len(ids))
        lut = pd.Series(np.arange(len(ids)), index=ids)
        return (torch.tensor(libs_s[self.library_col].map(lut).to_numpy()).to(torch.int64),
                torch.tensor(libs_g1[self.library_col].map(lut).to_numpy()).to(torch.int64))

    def make_g1_g2_training_data(self, cn_g1_states, cn_g1_reads, libs_g1):
        """pert_model.py:228-251: every G1/2 cell twice, rep = 0 then rep = 1."""
        libs = torch.cat([libs_g1, libs_g1], dim=0)
        states = torch.cat([cn_g1_states, cn_g1_states], dim=1)
        reads = torch.cat([cn_g1_reads, cn_g1_reads], dim=1)
        rep = torch.cat([torch.zeros(cn_g1_states.shape), torch.ones(cn_g1_states.shape)], dim=1)
        return states, reads, libs, rep

    def convert_rt_prior_units(self, rt_prior_profile):
        """pert_model.py:254-257 (the RT prior is parsed but never used by the model)."""
        return rt_prior_profile / max(rt_prior_profile)

    def build_trans_mat(self, cn):
        """pert_model.py:260-269 (unused by the reference's fits): eye + 1 plus the counts of
        state transitions between consecutive loci of every cell."""
        c = np.asarray(_np(cn)).astype(np.int64)
        prev, cur = c[:-1].reshape(-1), c[1:].reshape(-1)
        counts = np.bincount(prev * self.P + cur, minlength=self.P * self.P).reshape(self.P, self.P)
        return torch.eye(self.P, self.P) + 1 + torch.as_tensor(counts, dtype=torch.float32)

    def build_cn_prior(self, cn, weight=None):
        """pert_model.py:272-282: dense (loci, cells, P) eta, ones with eta[l, n, cn[l, n]] = weight."""
        w = self.cn_prior_weight if weight is None else weight
        return torch.as_tensor(prep.build_cn_prior(_np(cn).astype(np.int64), w, self.P).dense())

    def build_clone_cn_prior(self, cn, cn_df, cn_tensor, clone_cn_profiles):
        """pert_model.py:285-296: each cell (cn_df.columns) takes its clone's consensus
        profile (int64-truncated) as prior state; dense (loci, cells, P).  The profile is
        aligned to cn_df's loci by (chr, start) (the reference indexes it positionally)."""
        return torch.as_tensor(self._clone_prior(cn, cn_df.columns, clone_cn_profiles, loci=cn_df.index).dense())

    def _clone_prior(self, cn, cells, profiles, loci=None, keys=None, cell_range=None) -> EtaCodebook:
        inp = self._prepare()
        lc = inp.loci_chr if loci is None else np.asarray(loci.get_level_values(0)).astype(str)
        ls = inp.loci_start if loci is None else np.asarray(loci.get_level_values(1))
        return prep.build_clone_cn_prior(cn, np.asarray(cells), lc, ls, profiles, self.cn_prior_weight, self.P,
                                         self.cell_col, self.clone_col, keys=keys, cell_range=cell_range)

    def build_composite_cn_prior(self, cn, clone_cn_profiles, weight=1e5):
        """pert_model.py:299-361 on the S cells (cn = cn_s_reads_df); dense (loci, cells, P)."""
        return torch.as_tensor(self._composite_prior(clone_cn_profiles, weight).dense())

    def _composite_prior(self, profiles, weight=1e5) -> EtaCodebook:
        inp = self._prepare()
        return prep.build_composite_cn_prior(inp, self.cn_s, self.cn_g1, profiles, self.P, J=self.J, weight=weight,
                                             cell_col=self.cell_col, clone_col=self.clone_col,
                                             cn_state_col=self.cn_state_col)

    def manhattan_binarization(self, X, MEAN_GAP_THRESH=0.7, EARLY_S_SKEW_THRESH=0.2, LATE_S_SKEW_THRESH=-0.2):
        """pert_model.py:364-423 for one cell: (cell_rt, frac_rt)."""
        return prep.manhattan_binarization(X, MEAN_GAP_THRESH, EARLY_S_SKEW_THRESH, LATE_S_SKEW_THRESH)

    def guess_times(self, cn_s_reads, etas):
        """pert_model.py:426-457: (t_init, t_alpha_prior, t_beta_prior) as float32 tensors;
        ``etas`` is the dense (loci, cells, P) prior or an EtaCodebook."""
        states = etas.argmax_states() if isinstance(etas, EtaCodebook) else torch.argmax(etas, dim=2).numpy()
        t, a, b = self._guess_times(_np(cn_s_reads), states)
        return torch.as_tensor(t), torch.as_tensor(a), torch.as_tensor(b)

    def _guess_times(self, reads, cn_states):
        if self.tau_init_method == 'sklearn':
            return prep.guess_times(reads, cn_states, self.upsilon, self.n_jobs)
        return guess_times_batched(reads, cn_states, self.upsilon, device=self.device, n_threads=self.tau_threads)

    def make_gc_features(self, x):
        """pert_model.py:460-463: columns [x^K, ..., x, 1]."""
        x = x.unsqueeze(1)
        return torch.cat([x ** i for i in reversed(range(0, self.K + 1))], 1)

    def _build_etas(self, inp, profiles, cells: Optional[slice] = None) -> EtaCodebook:
        """pert_model.py:668-716 as a code book; ``cells``: only that contiguous range of the
        S cells (a rank's shard)."""
        m, P, w = self.cn_prior_method, self.P, self.cn_prior_weight
        L, N = inp.reads_s.shape
        sl = slice(0, N) if cells is None else cells
        if m == 'hmmcopy':
            return prep.build_cn_prior(inp.states_s[:, sl], w, P)
        if m == 'g1_clones':
            return self._clone_prior(self._raw_table("s"), inp.cells_s, profiles, keys=inp.keys_s, cell_range=cells)
        if m == 'diploid':
            return prep.diploid_prior(L, sl.stop - sl.start, w, P)
        if m not in ('g1_cells', 'g1_composite'):
            return prep.uniform_prior(L, sl.stop - sl.start, P)
        if m == 'g1_cells':
            etas = prep.build_g1_cells_prior(inp, self.cn_s, self.cn_g1, w, P, self.cell_col, self.clone_col)
        else:
            etas = self._composite_prior(profiles)
        return etas if cells is None else etas.cells(cells)

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
        if self.log_steps and logging.getLogger().isEnabledFor(logging.INFO):
            for i, loss in enumerate(losses):
                logging.info('step: {}, loss: {}'.format(i, loss))      # root logger, as :747
        if reason == 1:
            print('ELBO converged at iteration ' + str(len(losses) - 1))
        elif reason == 2:
            print('ELBO is NaN at iteration ' + str(len(losses) - 1))
        self.timings[label] = time.perf_counter() - t0
        self.iters[label] = len(losses)
        self.launched[label] = getattr(shard, "last_launched", len(losses))   # iterations queued
        return losses

    @staticmethod
    def _cells(init, sl, N):
        """The rank's slice of the per-cell entries of an init dict (entries made for the
        rank's cells only, init_params(cells=...), are taken as they are)."""
        out = {}
        for k, v in init.items():
            v = np.asarray(v)
            per_cell = k in ("expose_tau", "expose_u", "expose_betas") and v.shape[0] == N
            out[k] = v[sl] if per_cell else v
        return out

    # one-launch steps (pert_enum_step: pass, reductions, priors, Adam and the loss record in
    # one launch) where launch latency, not the pass, sets the step time: one rank and at most
    # this many cell.bins (the C1 stand-in, 400 cells x 271 bins); PERT_FUSED=0/1 forces it
    FUSED_MAX_CELLBINS = 1 << 21

    def _fused(self, kind, dd: "_Dist", n_cellbins: int) -> bool:
        mode = os.environ.get("PERT_FUSED", "auto")
        if mode in ("0", "1"):
            return mode == "1" and dd.world == 1
        return dd.world == 1 and kind != KIND_STEP1 and n_cellbins <= self.FUSED_MAX_CELLBINS

    def _shard(self, kind, dd: _Dist, reads, libs, init, eta=None, **kw):
        """PertShard over this rank's contiguous cell range of the fit."""
        N = reads.shape[1]
        s0, s1 = dd.bounds(N)
        sl = slice(s0, s1)
        kw.setdefault("fused", self._fused(kind, dd, reads.shape[0] * (s1 - s0)))
        if eta is not None and eta.codes.shape[1] == N and s1 - s0 != N:
            eta = eta.cells(sl)                 # (a code book of the rank's cells is taken as is)
        for k in ("cn_obs", "rep_obs"):
            if k in kw:
                kw[k] = np.asarray(kw[k])[:, sl]
        return PertShard(kind, np.ascontiguousarray(reads[:, sl]), self._inp.gc, np.asarray(libs)[sl], self.L,
                         self.P, self.K, self._cells(init, sl, N), eta=eta, device=self.device, lr=self.learning_rate,
                         dirichlet_mode=self.dirichlet_mode, is_root=dd.rank == 0, n_cells_total=N,
                         allreduce=dd.allreduce, comm=dd.comm, **kw)

    def _shard_pairs(self, dd: _Dist, reads_g, states_g, libs2, init):
        """Step 1's PertShard in pair mode over this rank's contiguous range of G1/2 cells:
        both copies of each of its cells (the copies of a cell never straddle ranks)."""
        NG = reads_g.shape[1]
        a, b = dd.bounds(NG)
        idx = np.r_[a:b, NG + a:NG + b]
        cells = {k: (np.asarray(v)[idx] if k in ("expose_tau", "expose_u", "expose_betas") else v)
                 for k, v in init.items()}
        return PertShard(KIND_STEP1, np.ascontiguousarray(reads_g[:, a:b]), self._inp.gc, np.asarray(libs2)[idx],
                         self.L, self.P, self.K, cells, cn_obs=np.ascontiguousarray(states_g[:, a:b]), paired=True,
                         device=self.device, lr=self.learning_rate, dirichlet_mode=self.dirichlet_mode,
                         is_root=dd.rank == 0, n_cells_total=2 * NG, allreduce=dd.allreduce, comm=dd.comm)

    def _decode(self, shard: PertShard, dd: _Dist):
        cn, rep = shard.decode()
        c = shard.constrained()
        cn = dd.gather_cells(cn.cpu().numpy())
        rep = dd.gather_cells(rep.cpu().numpy())
        for k in ("expose_tau", "expose_u"):
            c[k] = dd.gather_cells(np.asarray(c[k]))
        return cn, rep, c

    def run_pert_model(self):
        t_all = time.perf_counter()
        P, K = self.P, self.K
        # the device first: the library's communicator is made on the current device
        if self.device.type == "cuda" and self.device.index is not None:
            torch.cuda.set_device(self.device)
        dd = _Dist(self._group, device=self.device)
        # host work that only steps 2/3 need runs on a helper thread: the consensus profiles as
        # soon as the G1/2 table is sorted (while the S table is prepared), the step-2 prior and
        # tau initialisation while step 1 fits, then (during step 2) the step-3 prior and tau
        # initialisation -- device parts on a side stream
        from concurrent.futures import ThreadPoolExecutor
        # (the fit thread queues chunks of iterations by GIL-releasing C calls, 64 iterations
        # ahead of the device -- more than the interpreter's 5 ms switch interval lasts -- so the
        # helper's Python work does not starve the device, PertShard.run_svi)
        # Before the helper exists: the library scans of the tau initialiser's host path (a scan
        # on the helper, beside a GIL-holding library load on this thread, deadlocks the two:
        # tau_init.prepare_host_threads) and, with sklearn's public KMeans fallback, the BLAS
        # thread count held at one for the fit
        threads = contextlib.ExitStack()
        threads.enter_context(host_threads())
        helper = ThreadPoolExecutor(max_workers=1, thread_name_prefix="pert-prep")

        def on_device(fn, *a):
            # the HIP runtime's current device is per thread: the helper uses the fit's device
            if self.device.type != "cuda":
                return fn(*a)
            with torch.cuda.device(self.device):
                return fn(*a)

        def consensus(cn_g1, keys_g):
            t0 = time.perf_counter()
            prof = prep.consensus_clone_profiles(
                cn_g1, self.cn_state_col, clone_col=self.clone_col, cell_col=self.cell_col,
                chr_col=self.chr_col, start_col=self.start_col, cn_state_col=self.cn_state_col, keys=keys_g)
            return prof, time.perf_counter() - t0

        phases = self.timings.setdefault("phases", [])      # (phase, end time since the call began)
        phases.clear()

        def mark(name):
            phases.append((name, round(time.perf_counter() - t_all, 4)))

        try:
            # step 1's canonical pi trajectory (data independent, ~0.2 ms of host work per
            # iteration): computed on the helper while the fit thread prepares the inputs
            helper.submit(CanonicalPiBlock.precompute, P, self.learning_rate, self.max_iter_step1 + 1)
            fut_prof = []
            tic = time.perf_counter()
            inp = self._prepare(on_g1_sorted=lambda t, k: fut_prof.append(helper.submit(on_device, consensus, t, k)),
                                defer_sorted=True)
            if not fut_prof:                       # inputs prepared before this call: consensus now
                fut_prof.append(helper.submit(on_device, consensus, self.cn_g1, inp.keys_g))
            n_libs = self.L
            self.timings["prep"] = time.perf_counter() - tic
            # this rank's S / G1/2 cells (all of them on one rank): the priors, the tau
            # initialisers, the ploidy and the per-cell initial values are made for those only
            cells_s = slice(*dd.bounds(inp.reads_s.shape[1]))
            cells_g = slice(*dd.bounds(inp.reads_g.shape[1]))

            def priors():
                profiles, t_cons = fut_prof[0].result()         # ran earlier on this same thread
                t0 = time.perf_counter()
                etas = self._build_etas(inp, profiles, cells=cells_s if dd.world > 1 else None)
                t1 = time.perf_counter()
                # step 2's tau initialisation (:790), its device part on a side stream
                stream = torch.cuda.Stream(device=self.device) if self.device.type == "cuda" else None
                with (torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext()):
                    t_init, _, _ = self._guess_times(inp.reads_s[:, cells_s], etas.argmax_states())
                    if stream is not None:
                        stream.synchronize()
                self.timings["tau_init_s"] = dict(getattr(guess_times_batched, "last_timings", {}))
                return profiles, etas, t_init, (t_cons + t1 - t0, time.perf_counter() - t1)

            fut_priors = helper.submit(on_device, priors)

            # ---- step 1: G1/2 cells doubled, cn / rep observed (:718-774)
            # the doubled training set (make_g1_g2_training_data, :228-251) in pair mode: the
            # G1/2 columns stored once, rep 0 / rep 1 copies as cells [0, NG) / [NG, 2 NG)
            mean_g = np.mean(inp.reads_g, axis=0, dtype=np.float64)
            lb_g2 = np.concatenate([inp.libs_g, inp.libs_g])
            init1 = init_params(KIND_STEP1, None, lb_g2, n_libs, P, K, seed=self.seed, method=self.init_method,
                                mean_reads=np.concatenate([mean_g, mean_g]), n_bins=inp.reads_g.shape[0])
            mark("prep")
            s1 = self._shard_pairs(dd, inp.reads_g, inp.states_g, lb_g2, init1)
            self.timings["init_shard1"] = s1.init_timings
            mark("init_shard1")
            logging.info('STEP 1: Learning reads to CN bias from low variance cells.')
            losses_g = self._svi(s1, self.max_iter_step1, self.min_iter_step1, "step1")
            c1 = s1.constrained()
            lambda_fit = np.asarray(c1["expose_lambda"], dtype=np.float32)
            beta_means_fit = np.asarray(c1["expose_beta_means"], dtype=np.float32)
            self.step1_sites = {"lambda": lambda_fit, "beta_means": beta_means_fit}     # for inspection
            del s1
            mark("step1")

            # ---- step 2: S cells, enumerated (:776-830)
            tic = time.perf_counter()
            profiles, etas, t_init, (t_priors, t_guess) = fut_priors.result()
            self.t_init_s = t_init                 # step 2's tau initialisation (:790) of this rank's cells
            # wall time step 1 did not hide (the helper's own durations: timings["helper_*"])
            self.timings["guess_times_s"] = time.perf_counter() - tic
            self.timings["helper_priors"], self.timings["helper_guess_times_s"] = t_priors, t_guess
            mark("wait_priors")
            # (the helper runs its tasks in order: the two tau initialisers never share the pool)
            fut_prep3 = (helper.submit(on_device, self._prep_step3, inp, profiles, cells_g if dd.world > 1 else None)
                         if self.run_step3 else None)
            ploidy = etas.ploidy()
            init2 = init_params(KIND_STEP2, inp.reads_s, inp.libs_s, n_libs, P, K, ploidy=ploidy, t_init=t_init,
                                beta_means=beta_means_fit, seed=self.seed, method=self.init_method, cells=cells_s)
            s2 = self._shard(KIND_STEP2, dd, inp.reads_s, inp.libs_s, init2, eta=etas, lamb=float(lambda_fit[0]),
                             beta_means=beta_means_fit)
            self.timings["init_shard2"] = s2.init_timings
            mark("init_shard2")
            # the sorted copies of the input tables (packaging's) are built while step 2 runs in
            # the library (the fit thread waits in one GIL-free call): not beside the host work
            # before it, whose interpreter time they would take
            for t in (self._raw_table("s"), self._raw_table("g")):
                if isinstance(t, prep.DeferredTable):
                    t.start()
            logging.info('STEP 2: Jointly infer replication and CN states in high variance cells.')
            losses_s = self._svi(s2, self.max_iter, self.min_iter, "step2")
            mark("step2")
            tic = time.perf_counter()
            cn_map, rep_map, c2 = self._decode(s2, dd)
            trace_s = MapTrace(cn=cn_map, rep=rep_map, expose_u=c2["expose_u"], expose_rho=c2["expose_rho"],
                               expose_a=c2["expose_a"], expose_tau=c2["expose_tau"])
            cn_s_out, supp_s_out_df = self.package_s_output(
                self.cn_s, trace_s, self._axes(inp.cells_s, inp.keys_s), lambda_fit, losses_g, losses_s)
            self.timings["decode_package_s"] = time.perf_counter() - tic
            rho_fit = c2["expose_rho"]
            a_fit = c2["expose_a"]
            del s2
            mark("decode_package2")

            cn_g1_out = supp_g1_out_df = None
            if self.run_step3:
                # ---- step 3: G1 cells with rho, a frozen (:834-896)
                tic = time.perf_counter()
                etas2, t_init2, t_guess2 = fut_prep3.result()
                self.t_init_g = t_init2
                self.timings["helper_guess_times_g"] = t_guess2
                ploidy2 = etas2.ploidy()
                self.timings["prep_step3"] = time.perf_counter() - tic      # the part step 2 did not hide
                init3 = init_params(KIND_STEP3, inp.reads_g, inp.libs_g, n_libs, P, K, ploidy=ploidy2,
                                    t_init=t_init2, beta_means=beta_means_fit, seed=self.seed, method=self.init_method,
                                    cells=cells_g)
                s3 = self._shard(KIND_STEP3, dd, inp.reads_g, inp.libs_g, init3, eta=etas2, lamb=float(lambda_fit[0]),
                                 beta_means=beta_means_fit, rho_fixed=np.asarray(rho_fit).reshape(-1),
                                 a_fixed=float(np.asarray(a_fit)[0]))
                mark("init_shard3")
                logging.info('STEP 3: Running pre-trained S-phase model on low variance cells.')
                losses_s2 = self._svi(s3, self.max_iter_step3, self.min_iter_step3, "step3")
                mark("step3")
                tic = time.perf_counter()
                cn3, rep3, c3 = self._decode(s3, dd)
                trace_s2 = MapTrace(cn=cn3, rep=rep3, expose_u=c3["expose_u"], expose_rho=rho_fit, expose_a=a_fit,
                                    expose_tau=c3["expose_tau"])
                cn_g1_out, supp_g1_out_df = self.package_s_output(
                    self.cn_g1, trace_s2, self._axes(inp.cells_g, inp.keys_g), lambda_fit, losses_g, losses_s2)
                self.timings["decode_package_g"] = time.perf_counter() - tic
                del s3
                mark("decode_package3")
        except BaseException:
            # this rank failed: raise the abort word its peers' sharded loops poll, so they
            # return with CommError now instead of at the communicator's deadline
            if dd.comm is not None and dd.comm.status() == 0:
                dd.comm.abort()
            raise
        finally:
            # also when a fit or a helper task raised: no helper work outlives the call
            helper.shutdown(wait=True, cancel_futures=True)
            threads.close()
            dd.close()
        self.timings["total"] = time.perf_counter() - t_all
        return cn_s_out, supp_s_out_df, cn_g1_out, supp_g1_out_df

    def _prep_step3(self, inp, profiles, cells: Optional[slice] = None):
        """Step 3's clone prior on the G1/2 cells and their tau initialisation (:836-858), on
        the helper thread while step 2 fits: the device part of the initialiser on a side
        stream of its own.  ``cells``: this rank's G1/2 cells only (a sharded fit)."""
        stream = torch.cuda.Stream(device=self.device) if self.device.type == "cuda" else None
        ctx = torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext()
        with ctx:
            etas2 = self._clone_prior(self._raw_table("g"), inp.cells_g, profiles, keys=inp.keys_g, cell_range=cells)
            t0 = time.perf_counter()
            reads = inp.reads_g if cells is None else inp.reads_g[:, cells]
            t_init2, _, _ = self._guess_times(reads, etas2.argmax_states())
            if stream is not None:
                stream.synchronize()
            self.timings["tau_init_g"] = dict(getattr(guess_times_batched, "last_timings", {}))
        return etas2, t_init2, time.perf_counter() - t0

    # ------------------------------------------------------------------ outputs
    def package_s_output(self, cn_s, trace_s, cn_s_reads_df, lambda_fit, losses_g, losses_s):
        """pert_model.py:466-538: per (bin, cell) model_cn_state / model_rep_state, per cell
        model_tau / model_u, per bin model_rho -- the rows, row order and dtypes of the
        reference's melt + inner merges on (cell, chr, start) -- plus the supp frame of
        lambda, a and the loss traces.  ``trace_s``: a MapTrace (or anything with
        ``nodes[name]['value']``); ``cn_s_reads_df``: the (loci x cells) frame or a PivotAxes."""
        nodes = trace_s.nodes
        v = lambda k: _np(nodes[k]["value"])
        cells = np.asarray(cn_s_reads_df.columns)
        idx = cn_s_reads_df.index
        loci_chr = np.asarray(idx.get_level_values(0)).astype(str)
        loci_start = np.asarray(idx.get_level_values(1))
        keys = getattr(cn_s_reads_df, "keys", None)
        if keys is not None and not isinstance(keys, prep.TableKeys):
            keys = None                                   # a DataFrame's .keys is a method
        if keys is not None and prep._n_rows(keys) == len(cn_s) and keys.is_grid(cells, loci_chr, loci_start):
            ci = li = None                                # row i = (cell i // L, locus i % L)
        elif keys is not None and prep._n_rows(keys) == len(cn_s):
            ci, li = keys.row_positions(cells, loci_chr, loci_start)
        else:
            cell_index = pd.Index(cells.astype(str))
            locus_index = pd.MultiIndex.from_arrays([loci_chr, loci_start])
            ci = cell_index.get_indexer(cn_s[self.cell_col].astype(str).to_numpy())
            li = locus_index.get_indexer(pd.MultiIndex.from_arrays(
                [cn_s[self.chr_col].astype(str).to_numpy(), cn_s[self.start_col].to_numpy()]))
        model_cn, model_rep = v("cn"), v("rep")
        per_cell = lambda k: v(k).astype(np.float32).reshape(-1)
        if ci is None:
            base = cn_s
            L = len(loci_start)
            model = {
                'model_cn_state': prep.transpose_cast(model_cn, np.int64).reshape(-1),
                'model_rep_state': prep.transpose_cast(model_rep, np.float32).reshape(-1),
                'model_tau': np.repeat(per_cell("expose_tau"), L),
                'model_u': np.repeat(per_cell("expose_u"), L),
                'model_rho': np.tile(per_cell("expose_rho"), len(cells)),
            }
        else:
            keep = (ci >= 0) & (li >= 0)
            base = cn_s.loc[keep] if not keep.all() else cn_s
            ci, li = ci[keep], li[keep]
            model = {
                'model_cn_state': model_cn[li, ci].astype(np.int64),
                'model_rep_state': model_rep[li, ci].astype(np.float32),
                'model_tau': per_cell("expose_tau")[ci],
                'model_u': per_cell("expose_u")[ci],
                'model_rho': per_cell("expose_rho")[li],
            }
        # new columns side by side with the (sorted) input rows, without copying its blocks:
        # each inserted column is a block of its own (reset_index(drop=True) would deep-copy
        # the whole long table, and a concat consolidates every block of one dtype)
        out = base.copy(deep=False)
        out.index = pd.RangeIndex(len(out))
        for name, col in model.items():
            out[name] = col
        lam = float(_np(lambda_fit).reshape(-1)[0])
        a = float(v("expose_a").reshape(-1)[0])
        supp = pd.concat([
            pd.DataFrame({'param': ['model_lambda'], 'level': ['all'], 'value': [lam]}),
            pd.DataFrame({'param': ['model_a'], 'level': ['all'], 'value': [a]}),
            pd.DataFrame({'param': ['loss_g'] * len(losses_g), 'level': np.arange(len(losses_g)), 'value': losses_g}),
            pd.DataFrame({'param': ['loss_s'] * len(losses_s), 'level': np.arange(len(losses_s)), 'value': losses_s}),
        ], ignore_index=True)
        return out, supp
