"""reference scdna_replication_tools/compute_consensus_clone_profiles.py (:17-88).

``compute_consensus_clone_profiles`` with the median (the reference default) runs on
integer keys and one sort (prep.consensus_clone_profiles, pinned bit for bit to the
reference's own output by tests/golden/consensus_reference.npz); another ``aggfunc``
takes pandas' pivot_table over the same majority-ploidy rows."""
import numpy as np
import pandas as pd

from scdna_replication_tools_amd import prep


def add_cell_ploidies(cn, cell_col='cell_id', cn_state_col='state', ploidy_col='ploidy'):
    """:30-39: each row gets its cell's modal state (ties to the smallest, scipy.stats.mode)."""
    pl = prep.cell_ploidies(cn, cell_col=cell_col, cn_state_col=cn_state_col)
    cn[ploidy_col] = cn[cell_col].map(pl).astype(np.float64)
    return cn


def filter_ploidies(cn, clone_col='clone_id', ploidy_col='ploidy'):
    """:17-27: the rows of each clone's most frequent ploidy (row counts, ties to the smallest)."""
    return prep.filter_ploidies(cn, clone_col=clone_col, ploidy_col=ploidy_col).reset_index(drop=True)


def compute_consensus_clone_profiles(cn, col_name, clone_col='clone_id', cell_col='cell_id', chr_col='chr',
                                     start_col='start', cn_state_col='state', ploidy_col='ploidy', aggfunc=np.median):
    """:42-88: (loci x clones) consensus of ``col_name`` over each clone's majority-ploidy cells."""
    if aggfunc is np.median or aggfunc == "median":
        return prep.consensus_clone_profiles(cn, col_name, clone_col=clone_col, cell_col=cell_col, chr_col=chr_col,
                                             start_col=start_col, cn_state_col=cn_state_col)
    cn = cn[cn[clone_col] != 'None'].copy()
    if cn_state_col is not None:
        cn = filter_ploidies(add_cell_ploidies(cn, cell_col, cn_state_col, ploidy_col), clone_col, ploidy_col)
    return cn.pivot_table(index=[chr_col, start_col], columns=clone_col, values=col_name, aggfunc=aggfunc)


__all__ = ["compute_consensus_clone_profiles", "add_cell_ploidies", "filter_ploidies"]
