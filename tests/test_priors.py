"""CN prior (eta) builders against literal restatements of the reference's per-cell loops
(CPU): ``build_composite_cn_prior`` (pert_model.py:299-361) with ``compute_cell_corrs``
(normalize_by_cell.py:148-180), the ``g1_cells`` branch (:671-701), ``diploid`` (:708-712)
and the uniform fallback (:714-716).

The restatements below are the reference's pandas/scipy calls (merge per cell pair,
``scipy.stats.pearsonr``, ``sort_values(ascending=False)``, ``iloc[j]``, add_cell_ploidies +
filter_ploidies with scipy's mode).  Cases: J capped by the smallest clone, an off-ploidy
G1 cell dropped by the majority-ploidy filter, tied correlations (duplicate G1 read
profiles with different states, so the tie order shows in eta), a constant G1 profile
(NaN r, ranked last), and a clone left with fewer than J cells by the ploidy filter
(the reference raises IndexError; so does the build).
"""
import warnings

import numpy as np
import pandas as pd
import pytest
import torch
from scipy.stats import mode, pearsonr

from scdna_replication_tools_amd import prep

P = 13


# --------------------------------------------------------------------------- data
def _tables(seed=0, n_s=9, clones_g=(("A", 5), ("B", 3)), n_loci=40, tie=False, const=False, off_ploidy=True):
    """Long-form S / G1 tables: per clone a CN profile; reads ~ Poisson(30 * state) with a
    per-cell replication bump on the S cells."""
    rng = np.random.default_rng(seed)
    chroms = np.repeat(["1", "2", "X"], n_loci // 3 + 1)[:n_loci]
    starts = np.tile(np.arange(n_loci // 3 + 1) * 500000 + 1, 3)[:n_loci]
    prof = {"A": np.full(n_loci, 2), "B": np.r_[np.full(n_loci // 4, 3), np.full(n_loci - n_loci // 4, 2)]}

    def rows(cid, clone, states, reads):
        return pd.DataFrame(dict(cell_id=cid, chr=chroms, start=starts, gc=0.4 + 0.001 * np.arange(n_loci),
                                 library_id="L0", clone_id=clone, state=states, reads=reads))
    g = []
    k = 0
    for clone, n in clones_g:
        for i in range(n):
            st = prof[clone].copy()
            if off_ploidy and clone == "A" and i == 0:
                st = st * 2                                   # a tetraploid G1 cell in clone A
            st = np.where(rng.uniform(size=n_loci) < 0.05, st + 1, st)
            g.append(rows("g{:02d}".format(k), clone, st, rng.poisson(30 * st).astype(float)))
            k += 1
    if tie:                                                   # a duplicate read profile, other states
        dup = g[1].copy()
        dup["cell_id"] = "g{:02d}".format(k)
        dup["state"] = np.where(np.arange(n_loci) % 4 == 0, 4, dup["state"])
        g.append(dup)
        k += 1
    if const:                                                 # constant reads: pearson r = NaN
        c = g[2].copy()
        c["cell_id"] = "g{:02d}".format(k)
        c["reads"] = 55.0
        g.append(c)
    s = []
    for i in range(n_s):
        clone = "A" if i % 3 else "B"
        st = prof[clone]
        bump = 1 + (rng.uniform(size=n_loci) < 0.4)
        s.append(rows("s{:02d}".format(i), clone, st, rng.poisson(25 * st * bump).astype(float)))
    cat = lambda parts: pd.concat(parts, ignore_index=True).sample(frac=1.0, random_state=seed).reset_index(drop=True)
    return cat(s), cat(g)


# --------------------------------------------------------------------------- reference restatements
def _ref_cell_corrs(s_cell_cn, clone_cn_g1, s_cell_id, col):
    """normalize_by_cell.py:148-180."""
    s_col, g1_col = '{}_s'.format(col), '{}_g1'.format(col)
    s_cell_cn[s_col] = s_cell_cn[col]
    s_cell_cn = s_cell_cn.drop(columns=[col])
    parts = []
    for g1_cell_id, g1_cell_cn in clone_cn_g1.groupby('cell_id'):
        g1_cell_cn = g1_cell_cn[['chr', 'start', col]].copy()
        g1_cell_cn[g1_col] = g1_cell_cn[col]
        g1_cell_cn = g1_cell_cn.drop(columns=[col])
        merged = pd.merge(s_cell_cn, g1_cell_cn)
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            r, pval = pearsonr(merged[s_col].values, merged[g1_col].values)
        parts.append(pd.DataFrame({'s_cell_id': [s_cell_id], 'g1_cell_id': [g1_cell_id], 'pearson_r': [r],
                                   'pearson_pval': [pval]}))
    cell_corrs = pd.concat(parts, ignore_index=True)
    cell_corrs.sort_values(by=['pearson_r'], ascending=False, inplace=True)
    return cell_corrs


def _ref_ploidy_pool(cn_g1):
    """add_cell_ploidies + filter_ploidies (compute_consensus_clone_profiles.py:17-39)."""
    cn = cn_g1.copy().set_index('cell_id')
    for cell_id, group in cn.groupby('cell_id'):
        cn.loc[cell_id, 'ploidy'] = mode(group['state'], keepdims=True)[0][0]
    cn = cn.reset_index()
    pieces = []
    for clone_id, group in cn.groupby('clone_id'):
        keep = group.groupby('ploidy').size().idxmax()
        pieces.append(group[group['ploidy'] == keep].copy())
    return pd.concat(pieces, ignore_index=True)


def _ref_build_cn_prior(cn, weight):
    L, N = cn.shape
    etas = torch.ones(L, N, P)
    for i in range(L):
        for n in range(N):
            etas[i, n, int(cn[i, n].numpy())] = weight
    return etas


def _ref_composite(cn_s, cn_g1, cells, profiles, J=5, weight=1e5, col='reads'):
    """build_composite_cn_prior (pert_model.py:299-361)."""
    smallest = cn_g1[['cell_id', 'clone_id']].drop_duplicates().groupby('clone_id').size().min()
    J = min(J, smallest)
    pool = _ref_ploidy_pool(cn_g1)
    L = profiles.shape[0]
    etas = torch.ones(L, len(cells), P)
    for n, cell_id in enumerate(cells):
        cell_cn = cn_s.loc[cn_s['cell_id'] == cell_id]
        clone = cell_cn['clone_id'].values[0]
        clone_prof = torch.tensor(profiles[clone].values).to(torch.int64).to(torch.float32)
        clone_g1 = pool.loc[pool['clone_id'] == clone]
        psi = _ref_cell_corrs(cell_cn.copy(), clone_g1, cell_id, col)
        g1_cns = np.zeros((L, J))
        for j in range(J):
            gid = psi.iloc[j].g1_cell_id
            g1_cns[:, j] = clone_g1.loc[clone_g1['cell_id'] == gid]['state'].values
        for i in range(L):
            etas[i, n, int(clone_prof[i].numpy())] += weight * J * 2
            for j in range(J):
                etas[i, n, int(g1_cns[i, j])] += weight * (J - j)
    return etas


def _ref_g1_cells(cn_s, cn_g1, cells, weight=1e6, col='reads'):
    """The g1_cells branch (pert_model.py:671-701)."""
    L = cn_s.loc[cn_s['cell_id'] == cells[0]].shape[0]
    prior_in = torch.zeros(L, len(cells))
    for i, cell_id in enumerate(cells):
        cell_cn = cn_s.loc[cn_s['cell_id'] == cell_id]
        clone_g1 = cn_g1.loc[cn_g1['clone_id'] == cell_cn['clone_id'].values[0]]
        cell_cn = cell_cn[['chr', 'start', 'cell_id', col, 'state']]
        corrs = _ref_cell_corrs(cell_cn.copy(), clone_g1, cell_id, col)
        gid = corrs.iloc[0].g1_cell_id
        prior_in[:, i] = torch.tensor(clone_g1.loc[clone_g1['cell_id'] == gid]['state'].values).to(
            torch.int64).to(torch.float32)
    return _ref_build_cn_prior(prior_in, weight)


def _prepared(s, g):
    cn_s, cn_g1, inp = prep.process_input_data(s, g)
    prof = prep.consensus_clone_profiles(cn_g1, "state")
    return cn_s, cn_g1, inp, prof


# --------------------------------------------------------------------------- tests
@pytest.mark.parametrize("tie,const", [(False, False), (True, False), (False, True), (True, True)])
def test_composite_prior_matches_reference(tie, const):
    s, g = _tables(seed=1, tie=tie, const=const)
    cn_s, cn_g1, inp, prof = _prepared(s, g)
    got = prep.build_composite_cn_prior(inp, cn_s, cn_g1, prof, P).dense()
    ref = _ref_composite(cn_s, cn_g1, inp.cells_s, prof).numpy()
    np.testing.assert_array_equal(got, ref)


def test_composite_prior_caps_j_by_the_smallest_clone():
    s, g = _tables(seed=2, clones_g=(("A", 6), ("B", 2)), off_ploidy=False)
    cn_s, cn_g1, inp, prof = _prepared(s, g)
    got = prep.build_composite_cn_prior(inp, cn_s, cn_g1, prof, P, J=5).dense()
    np.testing.assert_array_equal(got, _ref_composite(cn_s, cn_g1, inp.cells_s, prof, J=5).numpy())
    # J = 2 (clone B): the consensus state carries 1 + 4e5, the two matches 2e5 and 1e5
    assert got.max() <= 1 + 1e5 * 2 * 2 + 2e5 + 1e5


def test_composite_prior_raises_like_reference_when_filter_leaves_too_few():
    # clone A: 3 cells counted for J (J -> 3), one of them off-ploidy -> 2 left for 3 matches
    s, g = _tables(seed=3, clones_g=(("A", 3), ("B", 4)), off_ploidy=True)
    cn_s, cn_g1, inp, prof = _prepared(s, g)
    with pytest.raises(IndexError):
        _ref_composite(cn_s, cn_g1, inp.cells_s, prof)
    with pytest.raises(IndexError):
        prep.build_composite_cn_prior(inp, cn_s, cn_g1, prof, P)


def test_composite_prior_uses_an_existing_ploidy_column():
    """The reference only adds ploidies when cn_g1 has no 'ploidy' column (:315-316)."""
    s, g = _tables(seed=4, off_ploidy=False)
    g["ploidy"] = np.where(g["cell_id"] == "g03", 4.0, 2.0)     # declared, not the modal state
    cn_s, cn_g1, inp, prof = _prepared(s, g)
    got = prep.build_composite_cn_prior(inp, cn_s, cn_g1, prof, P).dense()
    pool = cn_g1[cn_g1["cell_id"] != "g03"]
    match = prep.g1_cell_matches(inp, cn_s, cn_g1, 3, g1_pool=pool)
    assert not (np.asarray(inp.cells_g)[match] == "g03").any()
    assert got.shape == (len(inp.loci_start), len(inp.cells_s), P)


@pytest.mark.parametrize("tie,const", [(False, False), (True, True)])
def test_g1_cells_prior_matches_reference(tie, const):
    s, g = _tables(seed=5, tie=tie, const=const)
    cn_s, cn_g1, inp, prof = _prepared(s, g)
    got = prep.build_g1_cells_prior(inp, cn_s, cn_g1, 1e6, P).dense()
    ref = _ref_g1_cells(cn_s, cn_g1, inp.cells_s).numpy()
    np.testing.assert_array_equal(got, ref)


def test_cell_corrs_match_reference_table():
    s, g = _tables(seed=6, tie=True, const=True)
    cn_s, cn_g1, inp, prof = _prepared(s, g)
    cell = inp.cells_s[0]
    s_cell = cn_s.loc[cn_s["cell_id"] == cell]
    pool = cn_g1.loc[cn_g1["clone_id"] == s_cell["clone_id"].values[0]]
    got = prep.compute_cell_corrs(s_cell.copy(), pool, cell, col="reads")
    ref = _ref_cell_corrs(s_cell.copy(), pool, cell, "reads")
    pd.testing.assert_frame_equal(got, ref, check_exact=False, rtol=1e-12)


def test_rank_matches_pandas_sort_values_on_ties_and_nans():
    rng = np.random.default_rng(0)
    v = np.round(rng.normal(size=(50, 23)), 1)                 # many ties
    v[3, [2, 7]] = np.nan
    v[9, :] = np.nan
    got = prep.rank_desc_like_pandas(v)
    for r in range(v.shape[0]):
        want = pd.DataFrame({"x": v[r]}).sort_values(by=["x"], ascending=False).index.to_numpy()
        np.testing.assert_array_equal(got[r], want)


def test_diploid_and_uniform_priors_match_reference():
    L, N = 17, 6
    d = prep.diploid_prior(L, N, 1e6, P).dense()
    ref = _ref_build_cn_prior(torch.ones(L, N, P)[:, :, 0] * 2, 1e6)          # (:708-712)
    np.testing.assert_array_equal(d, ref.numpy())
    u = prep.uniform_prior(L, N, P)
    np.testing.assert_array_equal(u.dense(), (torch.ones(L, N, P) / P).numpy())   # (:714-716)
    # ploidy (pert_model.py:591-593): mean argmax of eta = 0 for the uniform prior
    assert (u.argmax_states() == 0).all() and (prep.diploid_prior(L, N, 1e6, P).argmax_states() == 2).all()
