"""Synthetic stand-ins for BASELINE.json's configs (test infrastructure).

configs[0] (inference_tutorial.ipynb, data/D1.0: absent from the reference snapshot,
SURVEY.md section 8) is replaced by a seeded simulator sample of the same shape: 400 S +
400 G1/2 cells x 271 bins, diploid (one clone), one library, ~183 reads per bin, in the
tutorial's columns (cell 8: cell_id, chr, start, end, gc, state, library_id,
true_reads_norm; clone_id on the G1/2 cells only).
"""
from __future__ import annotations

import numpy as np

C1_COLS_S = ['cell_id', 'chr', 'start', 'end', 'gc', 'state', 'library_id', 'true_reads_norm']
C1_COLS_G = ['cell_id', 'chr', 'start', 'end', 'gc', 'clone_id', 'state', 'library_id', 'true_reads_norm']


def c1_tables(seed: int = 0, n_cells: int = 400, n_bins: int = 271):
    """(temp_cn_s, temp_cn_g1, truth_s) as the tutorial builds them (cells 2 and 8)."""
    from scdna_replication_tools_amd.simulator import simulate, to_long_form
    sim = simulate(n_s=n_cells, n_g=n_cells, n_bins=n_bins, n_clones=1, num_reads=183 * n_bins, seed=seed)
    df_s, df_g = to_long_form(sim, input_col='true_reads_norm', n_libs=1)
    for df in (df_s, df_g):
        df['end'] = df['start'] + 500000 - 1
    truth = df_s[['cell_id', 'chr', 'start', 'true_somatic_cn', 'true_rep']].copy()
    return df_s[C1_COLS_S].copy(), df_g[C1_COLS_G].copy(), truth


def tutorial_scrt(temp_cn_s, temp_cn_g1, **extra):
    """inference_tutorial.ipynb cell 9, verbatim arguments."""
    from scdna_replication_tools.infer_scRT import scRT
    return scRT(temp_cn_s, temp_cn_g1, input_col='true_reads_norm', clone_col='clone_id', assign_col='state',
                rt_prior_col=None, cn_state_col='state', gc_col='gc', cn_prior_method='g1_clones', max_iter=200,
                **extra)


def input_digest(*frames) -> str:
    """SHA-256 of the tables' values (the fixture records which inputs it was made from)."""
    import hashlib
    h = hashlib.sha256()
    for f in frames:
        for c in f.columns:
            h.update(c.encode())
            h.update(np.ascontiguousarray(f[c].astype(str).to_numpy().astype("U")).tobytes())
    return h.hexdigest()[:16]


GENOME_KW = dict(input_col='reads', clone_col='clone_id', assign_col='copy', rt_prior_col=None, cn_state_col='state',
                 gc_col='gc', cn_prior_method='g1_clones')


def genome_tables(seed: int = 7, n_s: int = 64, n_g: int = 64):
    """configs[2]-style genome-length sample (test_gpu_chain's genome fixture): the full
    5,451-bin 500 kb grid, 3 clones, 1e6 reads per cell, two libraries; (cn_s, cn_g1, truth_s)."""
    from scdna_replication_tools_amd.simulator import simulate, to_long_form
    sim = simulate(n_s=n_s, n_g=n_g, n_clones=3, num_reads=1e6, seed=seed)
    df_s, df_g = to_long_form(sim, n_libs=2)
    truth = df_s[['cell_id', 'chr', 'start', 'true_somatic_cn', 'true_rep']].copy()
    keep_s = ['cell_id', 'chr', 'start', 'end', 'gc', 'state', 'copy', 'reads', 'library_id', 'clone_id']
    keep_s = [c for c in keep_s if c in df_s.columns]
    keep_g = [c for c in keep_s if c in df_g.columns]
    return df_s[keep_s].copy(), df_g[keep_g].copy(), truth


def genome_scrt(cn_s, cn_g1, **extra):
    """The reference's entry point with its defaults (max_iter 2000, min_iter 100, rel_tol
    1e-6, steps 1 / 3 at half) on the genome-length sample, g1_clones prior."""
    from scdna_replication_tools.infer_scRT import scRT
    return scRT(cn_s, cn_g1, **GENOME_KW, **extra)
