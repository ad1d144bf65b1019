"""Drop-in ``scRT`` orchestrator (reference scdna_replication_tools/infer_scRT.py:25-168),
PERT level only.

``scRT(cn_s, cn_g1, ...).infer(level='pert')`` (or 'pyro') computes the consensus clone
profiles of ``assign_col``, assigns every S-phase cell to its best-correlated clone
(assign_s_to_clones.py:49-79, vectorised) and runs ``pert_infer_scRT`` on the GPU.
When ``clone_col`` is None the G1/2 cells are first clustered by KMeans + BIC
(cncluster.kmeans_cluster, infer_scRT.py:129-138).  The deterministic 'cell' / 'clone' /
'bulk' levels are outside this build's scope and raise.
"""
from __future__ import annotations

import numpy as np
import pandas as pd

from . import prep
from .cncluster import kmeans_cluster
from .pert_model import pert_infer_scRT


def assign_s_to_clones(s_phase_cells: pd.DataFrame, clone_df: pd.DataFrame, col_name='reads',
                       clone_col='clone_id', cell_col='cell_id', chr_col='chr', start_col='start'):
    """assign_s_to_clones.py:49-79: every S cell gets the clone whose consensus profile
    has the highest Pearson r with the cell's ``col_name`` over the shared loci."""
    # per-cell blocks (the concatenated per-cell tables of the tutorials): the pivot is a
    # transpose of the blocks and every row's cell is its block's -- no per-row hashing
    lay = prep._block_layout(s_phase_cells, cell_col, chr_col, start_col, col_name)
    # a new frame over the same column blocks (the reference mutates and returns its argument;
    # the new columns below are set on this frame only)
    s = s_phase_cells.copy(deep=False)
    chc = s[chr_col]
    if lay is not None and chc.dtype == object and all(isinstance(v, str) for v in chc.to_numpy()[:lay[1]]):
        pass             # every block holds block 0's label objects (_block_layout): already str
    else:
        s[chr_col] = chc.astype(str)
    clone_df = clone_df.copy()
    if set([chr_col, start_col]).issubset(set(clone_df.columns)):
        clone_df = clone_df.set_index([chr_col, start_col])
    row_cell = None
    if lay is not None:
        B, L, bp, q, ch0 = lay
        cells = np.ascontiguousarray(s[cell_col].to_numpy())[::L][bp]
        # float64 like the general pivot and the reference's pearsonr: the block pivot keeps an
        # integer column in float32, where the centring and norms would round differently
        piv = prep.Pivot(cells, np.array(prep.CHR_ORDER, dtype=object)[ch0[q]], s[start_col].to_numpy()[:L][q],
                         prep._block_pivot(s[col_name].to_numpy(), B, L, bp, q).astype(np.float64, copy=False))
        pos = np.empty(B, np.int64)
        pos[bp] = np.arange(B)                     # block (table order) -> sorted cell index
        row_cell = np.repeat(pos, L)
    else:
        piv = prep.pivot_cells_by_loci(s, col_name, cell_col, chr_col, start_col)
    cidx = pd.MultiIndex.from_arrays([clone_df.index.get_level_values(0).astype(str),
                                      clone_df.index.get_level_values(1)])
    li = cidx.get_indexer(pd.MultiIndex.from_arrays([piv.loci_chr.astype(str), piv.loci_start]))
    prof = clone_df.to_numpy(np.float64)

    def cell_r(n):
        v = piv.values[:, n]
        ok = (li >= 0) & np.isfinite(v)
        x = v[ok]
        Y = prof[li[ok]]
        okc = ~np.isnan(Y).any(axis=1)          # merged_df.dropna(): NaN rows only (inf stays)
        x, Y = x[okc], Y[okc]
        xc = x - x.mean()
        Yc = Y - Y.mean(0)
        with np.errstate(invalid="ignore", divide="ignore"):
            return (xc @ Yc) / (np.linalg.norm(xc) * np.linalg.norm(Yc, axis=0))

    def pick(r):
        # Series.argmax (:71): first maximum, NaN skipped; all NaN (a constant profile) gives
        # -1 in the pandas the reference ran on, i.e. the last clone
        return int(np.nanargmax(r)) if np.isfinite(r).any() else -1

    n_cells = piv.values.shape[1]
    picks = None
    if n_cells and np.all(li >= 0) and np.isfinite(prof).all() and np.isfinite(piv.values).all() and prof.shape[1] > 1:
        # every cell shares every locus: all correlations as one product; a cell whose top two
        # are within 1e-9 (relative) of each other, or any non-finite r, takes the per-cell
        # arithmetic above, so the picks are the per-cell loop's
        Y = prof[li]
        Yc = Y - Y.mean(0)
        X = piv.values
        Xc = X - X.mean(0)
        with np.errstate(invalid="ignore", divide="ignore"):
            R = (Xc.T @ Yc) / (np.linalg.norm(Xc, axis=0)[:, None] * np.linalg.norm(Yc, axis=0)[None, :])
        top2 = np.sort(R, axis=1)[:, -2:]
        close = ~np.isfinite(R).all(axis=1) | (np.abs(top2[:, 1] - top2[:, 0]) <= 1e-9 * np.abs(top2[:, 1]))
        picks = np.argmax(R, axis=1)
        for n in np.flatnonzero(close):
            picks[n] = pick(cell_r(n))
    best = [clone_df.columns[int(p)] for p in picks] if picks is not None else \
        [clone_df.columns[pick(cell_r(n))] for n in range(n_cells)]
    if row_cell is not None:
        # the per-cell labels' dtype as infer_objects finds it for the rows (the same set of
        # values), then one gather per row
        per_cell = pd.Series(np.asarray(best, dtype=object)).infer_objects().to_numpy()
        s[clone_col] = pd.Series(per_cell[row_cell], index=s.index)
    else:
        lut = dict(zip(piv.cells, best))
        s[clone_col] = s[cell_col].astype(str).map(lut)
    return s


def consensus_profiles(cn_g1: pd.DataFrame, col_name, clone_col='clone_id', cell_col='cell_id', chr_col='chr',
                       start_col='start', cn_state_col='state') -> pd.DataFrame:
    """compute_consensus_clone_profiles (infer_scRT.py:140-141) of the G1/2 table.  A per-cell
    block table is sorted by (cell, chr, start) with one gather per column into a temporary copy
    (the caller's table keeps its row order) and handed over with its RegularKeys, which takes
    the consensus' block path (no per-row hashing of the labels, identical result)."""
    lay = prep._block_layout(cn_g1, cell_col, chr_col, start_col, None)
    if lay is not None and cn_state_col is not None and cn_state_col in cn_g1.columns:
        L = lay[1]
        # the medians straight from the table's blocks: no sorted copy of the table
        prof = prep.consensus_from_blocks(cn_g1, lay, col_name, clone_col=clone_col, chr_col=chr_col,
                                          start_col=start_col, cn_state_col=cn_state_col)
        if prof is None:
            out, keys, _, _ = prep._block_table(cn_g1, lay, None, col_name, cn_state_col, cell_col, chr_col, start_col)
            prof = prep.consensus_clone_profiles(out, col_name, clone_col=clone_col, cell_col=cell_col,
                                                 chr_col=chr_col, start_col=start_col, cn_state_col=cn_state_col,
                                                 keys=keys)
        # the caller's chromosome labels (the consensus carries them as CHR_ORDER strings):
        # integer labels stay integers, a categorical column keeps its own categories; sorted
        # as pivot_table sorts them.  Every block holds the same loci: the first block's labels
        # are all the labels there are.
        col = cn_g1[chr_col]
        lab = {str(v): v for v in pd.unique(col.iloc[:L].dropna())}
        idx = prof.index
        vals = [lab.get(str(v), v) for v in idx.get_level_values(0)]
        lev0 = pd.Categorical(vals, dtype=col.dtype) if isinstance(col.dtype, pd.CategoricalDtype) else pd.Index(vals)
        prof.index = pd.MultiIndex.from_arrays([lev0, idx.get_level_values(1)], names=idx.names)
        return prof.sort_index()
    return prep.consensus_clone_profiles(cn_g1, col_name, clone_col=clone_col, cell_col=cell_col, chr_col=chr_col,
                                         start_col=start_col, cn_state_col=cn_state_col)


class scRT:
    def __init__(self, cn_s, cn_g1, input_col='reads', assign_col='copy', library_col='library_id', ploidy_col='ploidy',
                 cell_col='cell_id', cn_state_col='state', chr_col='chr', start_col='start', gc_col='gc',
                 rv_col='rt_value', rs_col='rt_state', frac_rt_col='frac_rt', clone_col='clone_id', rt_prior_col='mcf7rt',
                 cn_prior_method='hmmcopy', col2='rpm_gc_norm', col3='temp_rt', col4='changepoint_segments', col5='binary_thresh',
                 max_iter=2000, min_iter=100, max_iter_step1=None, min_iter_step1=None, max_iter_step3=None, min_iter_step3=None,
                 cn_prior_weight=1e6, learning_rate=0.05, rel_tol=1e-6, cuda=False, seed=0, P=13, K=4, J=5, upsilon=6,
                 run_step3=True, **engine_kwargs):
        self.cn_s = cn_s
        self.cn_g1 = cn_g1
        self.input_col = input_col
        self.assign_col = assign_col
        self.clone_col = clone_col
        self.library_col = library_col
        self.cell_col = cell_col
        self.cn_state_col = cn_state_col
        self.chr_col = chr_col
        self.start_col = start_col
        self.gc_col = gc_col
        self.ploidy_col = ploidy_col
        self.rt_prior_col = rt_prior_col
        self.rv_col = rv_col
        self.rs_col = rs_col
        self.frac_rt_col = frac_rt_col
        self.col2, self.col3, self.col4, self.col5 = col2, col3, col4, col5
        self.clone_profiles = None
        self.bulk_cn = None
        self.manhattan_df = None
        self.cn_prior_method = cn_prior_method
        self.cn_prior_weight = cn_prior_weight
        self.learning_rate = learning_rate
        self.max_iter = max_iter
        self.min_iter = min_iter
        self.rel_tol = rel_tol
        self.cuda = cuda
        self.seed = seed
        self.P = P
        self.K = K
        self.J = J
        self.upsilon = upsilon
        self.run_step3 = run_step3
        self.max_iter_step1 = int(self.max_iter / 2) if max_iter_step1 is None else max_iter_step1
        self.min_iter_step1 = int(self.min_iter / 2) if min_iter_step1 is None else min_iter_step1
        self.max_iter_step3 = int(self.max_iter / 2) if max_iter_step3 is None else max_iter_step3
        self.min_iter_step3 = int(self.min_iter / 2) if min_iter_step3 is None else min_iter_step3
        self.engine_kwargs = engine_kwargs

    def infer(self, level='pert'):
        """infer_scRT.py:108-124."""
        supp_s_out_df = pd.DataFrame({})
        supp_g1_out_df = pd.DataFrame({})
        cn_g1_out = pd.DataFrame({})
        if level in ('pyro', 'pert'):
            self.cn_s, supp_s_out_df, cn_g1_out, supp_g1_out_df = self.infer_pert_model()
        elif level in ('cell', 'clone', 'bulk'):
            raise NotImplementedError("level='{}' (deterministic non-PERT heuristics) is outside this build's "
                                      "scope; use level='pert'".format(level))
        else:
            raise ValueError(level)
        return self.cn_s, supp_s_out_df, cn_g1_out, supp_g1_out_df

    def infer_pert_model(self):
        """infer_scRT.py:127-168."""
        model = self._pert_model()
        self.model = model
        return model.run_pert_model()

    def _pert_model(self) -> pert_infer_scRT:
        """infer_scRT.py:127-161: clustering (clone_col None), consensus clone profiles of
        assign_col, S-phase cells assigned to clones, then the PERT model object."""
        if self.clone_col is None:
            # no clone labels: KMeans + BIC over the G1/2 cells' assign_col profiles (:129-138)
            piv = prep.pivot_any(self.cn_g1, self.assign_col, self.cell_col, self.chr_col, self.start_col)
            g1_mat = pd.DataFrame(piv.values, columns=pd.Index(piv.cells, name=self.cell_col),
                                  index=pd.MultiIndex.from_arrays([piv.loci_chr, piv.loci_start],
                                                                  names=[self.chr_col, self.start_col]))
            clusters = kmeans_cluster(g1_mat, max_k=20, device=self.engine_kwargs.get("device"))
            self.clusters = clusters
            # pd.merge(cn_g1, clusters, on=cell_col) for an inner join on a complete cluster table
            cid = clusters["cluster_id"].to_numpy().astype(np.int64)
            lay = prep._block_layout(self.cn_g1, self.cell_col, self.chr_col, self.start_col, None)
            row_cl = None
            if lay is not None:
                # per-cell blocks: a row's cell is its block's (no per-row label lookup)
                B, L = lay[0], lay[1]
                heads = np.ascontiguousarray(self.cn_g1[self.cell_col].to_numpy())[::L]
                ci = pd.Index(clusters["cell_id"].to_numpy()).get_indexer(heads)
                if (ci >= 0).all():
                    row_cl = np.repeat(cid[ci], L)
            if row_cl is not None:
                self.cn_g1 = self.cn_g1.copy(deep=False)
                self.cn_g1["cluster_id"] = row_cl
            else:
                lut = pd.Series(cid, index=clusters["cell_id"].to_numpy())
                self.cn_g1 = self.cn_g1.assign(cluster_id=self.cn_g1[self.cell_col].map(lut))
                self.cn_g1 = self.cn_g1[self.cn_g1["cluster_id"].notna()]
                self.cn_g1["cluster_id"] = self.cn_g1["cluster_id"].astype(np.int64)
            self.clone_col = 'cluster_id'
        self.clone_profiles = consensus_profiles(
            self.cn_g1, self.assign_col, clone_col=self.clone_col, cell_col=self.cell_col, chr_col=self.chr_col,
            start_col=self.start_col, cn_state_col=self.cn_state_col)
        self.cn_s = assign_s_to_clones(self.cn_s, self.clone_profiles, col_name=self.assign_col,
                                       clone_col=self.clone_col, cell_col=self.cell_col, chr_col=self.chr_col,
                                       start_col=self.start_col)
        model = pert_infer_scRT(
            self.cn_s, self.cn_g1, input_col=self.input_col, gc_col=self.gc_col, rt_prior_col=self.rt_prior_col,
            clone_col=self.clone_col, cell_col=self.cell_col, library_col=self.library_col,
            assign_col=self.assign_col, chr_col=self.chr_col, start_col=self.start_col,
            cn_state_col=self.cn_state_col, rs_col=self.rs_col, frac_rt_col=self.frac_rt_col,
            cn_prior_method=self.cn_prior_method, cn_prior_weight=self.cn_prior_weight,
            learning_rate=self.learning_rate, max_iter=self.max_iter, min_iter=self.min_iter, rel_tol=self.rel_tol,
            min_iter_step1=self.min_iter_step1, min_iter_step3=self.min_iter_step3,
            max_iter_step1=self.max_iter_step1, max_iter_step3=self.max_iter_step3, cuda=self.cuda, seed=self.seed,
            P=self.P, K=self.K, J=self.J, upsilon=self.upsilon, run_step3=self.run_step3, **self.engine_kwargs)
        return model
