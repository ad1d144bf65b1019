"""``assign_s_to_clones`` (CPU) against a literal restatement of the reference's
``clone_correlations`` / ``assign_s_to_clones`` (assign_s_to_clones.py:18-79, called at
infer_scRT.py:147-148 on inference_tutorial cell 9's path).

The restatement keeps the reference's pandas calls one for one; the only edit is
``DataFrame.items()`` for ``iteritems()`` (removed in pandas 2).  Cases: inf / NaN read
values in a cell, loci missing from the clone profiles, a NaN inside one clone profile,
a constant clone profile (r = NaN for that clone), a constant cell profile (r = NaN for
every clone: pandas' all-NaN ``argmax`` gives -1, the last clone), tied r (two identical
clone profiles: first maximum), string and integer clone ids, profiles given with chr /
start columns or as a (chr, start) index.
"""
import warnings

import numpy as np
import pandas as pd
import pytest
from scipy.stats import pearsonr

from scdna_replication_tools_amd.infer_scRT import assign_s_to_clones


def _ref_clone_correlations(clone_df, cell_cn, col_name='reads'):
    """assign_s_to_clones.py:18-46."""
    df = cell_cn[col_name]
    df.replace([np.inf, -np.inf], np.nan, inplace=True)
    df.dropna(inplace=True)
    merged_df = pd.merge(df, clone_df, left_index=True, right_index=True)
    merged_df.dropna(inplace=True)
    clone_df = merged_df.drop(columns=[col_name])
    clone_corrs = {}
    for clone_id, clone_cn in clone_df.items():                 # iteritems() in pandas < 2
        r, pval = pearsonr(merged_df[col_name], clone_cn)
        clone_corrs[clone_id] = [r, pval]
    return pd.DataFrame(clone_corrs)


def _ref_assign(s_phase_cells, clone_df, col_name='reads', clone_col='clone_id', cell_col='cell_id', chr_col='chr',
                start_col='start'):
    """assign_s_to_clones.py:49-79."""
    s_phase_cells[chr_col] = s_phase_cells[chr_col].astype(str)
    clone_idx = [chr_col, start_col]
    if set(clone_idx).issubset(set(clone_df.columns)):
        clone_df.set_index(clone_idx, inplace=True)
    for cell_id, cell_cn in s_phase_cells.groupby(cell_col):
        temp_cell_cn = cell_cn.set_index(clone_idx).copy()
        copy_corrs = _ref_clone_correlations(clone_df, temp_cell_cn, col_name)
        temp_idx = copy_corrs.iloc[0].argmax()
        best_clone = clone_df.columns[temp_idx]
        s_phase_cells.loc[cell_cn.index, clone_col] = best_clone
    return s_phase_cells


CHRS = ["1", "2", "X"]


def _loci(n_per_chr=40):
    return [(c, 500000 * i) for c in CHRS for i in range(n_per_chr)]


def _clones(ids, loci, rng, tie=False, nan_in=None, const=None, as_columns=True):
    """Consensus profiles (loci x clones): piecewise-constant copy numbers."""
    prof = {}
    for k, cid in enumerate(ids):
        v = np.full(len(loci), 2.0) + rng.normal(0, 0.05, len(loci))
        seg = rng.integers(0, len(loci) - 20)
        v[seg:seg + 20] += 1 + k
        prof[cid] = v
    if tie:                                     # an exact duplicate of the first clone, listed later
        prof[ids[-1]] = prof[ids[0]].copy()
    if nan_in is not None:
        prof[nan_in][3] = np.nan
    if const is not None:
        prof[const] = np.full(len(loci), 2.0)
    df = pd.DataFrame(prof, index=pd.MultiIndex.from_tuples(loci, names=["chr", "start"]))
    return df.reset_index() if as_columns else df


def _cells(clone_prof, loci, n_cells, rng, clone_ids, inf_nan=True, drop_loci=0, constant_cell=None):
    rows = []
    prof = clone_prof.set_index(["chr", "start"]) if "chr" in clone_prof.columns else clone_prof
    for n in range(n_cells):
        truth = clone_ids[n % len(clone_ids)]
        mu = np.nan_to_num(prof[truth].to_numpy(), nan=2.0) * rng.uniform(0.9, 1.6, len(loci))
        v = mu + rng.normal(0, 0.3, len(loci))
        if constant_cell is not None and n == constant_cell:
            v = np.full(len(loci), 3.0)
        keep = np.ones(len(loci), bool)
        if drop_loci:
            keep[rng.choice(len(loci), drop_loci, replace=False)] = False
        for i, (c, st) in enumerate(loci):
            if keep[i]:
                rows.append({"cell_id": "cell_S_{}".format(n), "chr": c, "start": st, "end": st + 499999,
                             "copy": v[i]})
        if inf_nan and n % 3 == 0:
            rows[-2]["copy"] = np.inf
            rows[-5]["copy"] = np.nan
    df = pd.DataFrame(rows)
    return df.sample(frac=1.0, random_state=int(rng.integers(1 << 30))).reset_index(drop=True)


def _compare(s, clone_df, **kw):
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")                  # ConstantInputWarning, all-NaN argmax FutureWarning
        ref = _ref_assign(s.copy(), clone_df.copy(), col_name="copy", **kw)
        got = assign_s_to_clones(s.copy(), clone_df.copy(), col_name="copy", **kw)
    col = kw.get("clone_col", "clone_id")
    a = got.set_index(["cell_id", "chr", "start"])[col]
    b = ref.set_index(["cell_id", "chr", "start"])[col].reindex(a.index)
    assert len(got) == len(ref)
    assert (a.to_numpy() == b.to_numpy()).all(), pd.DataFrame({"got": a, "ref": b})[a.to_numpy() != b.to_numpy()]
    return got


@pytest.mark.parametrize("ids", [["A", "B", "C"], [0, 1, 2, 3]])
@pytest.mark.parametrize("as_columns", [True, False])
def test_assign_matches_reference_loop(ids, as_columns):
    rng = np.random.default_rng(5 if as_columns else 6)
    loci = _loci()
    prof = _clones(ids, loci, rng, as_columns=as_columns)
    s = _cells(prof, loci, 24, rng, ids)
    got = _compare(s, prof)
    # the assignment recovers the simulated clones
    truth = {"cell_S_{}".format(n): ids[n % len(ids)] for n in range(24)}
    first = got.drop_duplicates("cell_id").set_index("cell_id")["clone_id"]
    assert all(first[c] == truth[c] for c in first.index)


def test_assign_missing_loci_nan_profile_and_constant_profiles():
    """Loci absent from the profiles (and from some cells), a NaN in one profile (its locus
    leaves every clone's correlation), a constant clone, and a constant cell."""
    rng = np.random.default_rng(11)
    ids = ["A", "B", "C", "D"]
    loci = _loci()
    prof = _clones(ids, loci, rng, nan_in="B", const="D")
    s = _cells(prof, loci, 15, rng, ids[:3], drop_loci=4, constant_cell=7)
    prof = prof.drop(index=[5, 17, 60]).reset_index(drop=True)           # loci missing from the profiles
    got = _compare(s, prof)
    # the constant cell: every r is NaN, the reference's argmax gives -1 -> the last clone
    assert set(got.loc[got.cell_id == "cell_S_7", "clone_id"]) == {"D"}


def test_assign_tied_correlations_take_first_clone():
    rng = np.random.default_rng(2)
    ids = ["A", "B", "C"]
    loci = _loci()
    prof = _clones(ids, loci, rng, tie=True)                            # C == A exactly
    s = _cells(prof, loci, 12, rng, ["A", "B"], inf_nan=False)
    got = _compare(s, prof)
    assert "C" not in set(got["clone_id"])


@pytest.mark.parametrize("ids", [["A", "B", "C"], [0, 1, 2]])
def test_assign_per_cell_block_table_matches_reference_loop(ids):
    """The per-cell-block table of the tutorials (each cell's rows contiguous, the same loci in
    every cell): the block-transpose pivot gives the reference loop's assignment for every row
    and the same column dtype as the general path (rows shuffled)."""
    from scdna_replication_tools_amd import prep
    rng = np.random.default_rng(11)
    loci = _loci()
    prof = _clones(ids, loci, rng)
    s = _cells(prof, loci, 30, rng, ids, inf_nan=False)
    s = s.sort_values(["cell_id", "chr", "start"], kind="stable").reset_index(drop=True)
    s["cell_id"] = s["cell_id"].map({c: c for c in s["cell_id"].unique()})   # one str object per cell
    assert prep._block_layout(s, "cell_id", "chr", "start", "copy") is not None
    got = _compare(s, prof)
    general = assign_s_to_clones(s.sample(frac=1.0, random_state=3).reset_index(drop=True), prof.copy(),
                                 col_name="copy")
    assert got["clone_id"].dtype == general["clone_id"].dtype


def test_assign_block_table_integer_column_in_float64():
    """An integer read-count column (the default col_name='reads') on the per-cell-block
    path: the correlations run in float64 like the general path and the reference, so
    near-tied clones are assigned alike."""
    from scdna_replication_tools_amd import prep
    rng = np.random.default_rng(23)
    ids = ["A", "B", "C"]
    loci = _loci()
    prof = _clones(ids, loci, rng)
    s = _cells(prof, loci, 30, rng, ids, inf_nan=False)
    s["reads"] = np.round(s["copy"].to_numpy() * 1e5).astype(np.int64)    # large counts: fp32 would round
    s = s.sort_values(["cell_id", "chr", "start"], kind="stable").reset_index(drop=True)
    s["cell_id"] = s["cell_id"].map({c: c for c in s["cell_id"].unique()})   # one str object per cell
    assert prep._block_layout(s, "cell_id", "chr", "start", "reads") is not None
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        ref = _ref_assign(s.copy(), prof.copy(), col_name="reads")
        got = assign_s_to_clones(s.copy(), prof.copy(), col_name="reads")
    assert (got["clone_id"].to_numpy() == ref["clone_id"].to_numpy()).all()


def test_assign_all_shared_loci_product_path_near_ties():
    """Every cell on every profile locus, no missing values: the correlations come from one
    matrix product; clones within 1e-9 of each other (a near-duplicate listed later) take the
    per-cell arithmetic, so the picks are the reference loop's."""
    from scdna_replication_tools_amd import prep
    rng = np.random.default_rng(31)
    ids = ["A", "B", "C", "D"]
    loci = _loci()
    prof = _clones(ids, loci, rng)
    prof["D"] = prof["A"] + rng.normal(0, 1e-8, len(loci))               # near-ties with A (r within ~1e-9)
    s = _cells(prof, loci, 60, rng, ids[:3], inf_nan=False)
    s = s.sort_values(["cell_id", "chr", "start"], kind="stable").reset_index(drop=True)
    s["cell_id"] = s["cell_id"].map({c: c for c in s["cell_id"].unique()})
    assert prep._block_layout(s, "cell_id", "chr", "start", "copy") is not None
    _compare(s, prof)
    _compare(s.sample(frac=1.0, random_state=1).reset_index(drop=True), prof)   # the general pivot
