"""Host prep (prep.py) against plain-pandas restatements of the reference's own code
paths (pert_model.py:133-225, compute_consensus_clone_profiles.py:17-88,
pert_model.py:272-296), on shuffled long tables with NaNs, several libraries and
chromosomes in non-lexicographic order.  CPU only."""
import numpy as np
import pandas as pd
import pytest

from scdna_replication_tools_amd import prep

CHR = [str(i + 1) for i in range(22)] + ["X", "Y"]


def _table(n_cells=7, prefix="c", seed=0, chroms=("1", "2", "10", "X"), per_chr=6, n_libs=2, nan_locus=False,
           order="shuffled", shared=False):
    rng = np.random.default_rng(seed)
    rows = []
    for i in range(n_cells):
        for ch in chroms:
            for j in range(per_chr):
                rows.append(dict(cell_id="{}{}".format(prefix, (i * 7919) % 1000), chr=ch, start=j * 500000 + 1,
                                 gc=0.3 + 0.01 * j + 0.001 * CHR.index(ch), library_id="L{}".format(i % n_libs),
                                 state=int(rng.integers(1, 5)), reads=float(rng.integers(0, 300)),
                                 clone_id="AB"[i % 2], copy=float(rng.uniform(1, 4)),
                                 note="n{}".format(j % 3)))         # a label that varies within a cell
    df = pd.DataFrame(rows)
    if order == "shuffled":
        df = df.sample(frac=1.0, random_state=seed).reset_index(drop=True)
    else:
        # grouped by cell like concatenated per-cell HMMcopy tables, cells in a random order;
        # 'cells_split': one cell's block cut in two and moved apart (leaves the block path);
        # 'cells_unsorted': EVERY cell's loci in one shuffled order (the block path)
        blocks = [b for _, b in df.groupby("cell_id", sort=False)]
        perm = np.random.default_rng(seed).permutation(len(blocks))
        blocks = [blocks[i] for i in perm]
        if order == "cells_split":
            b = blocks.pop(0)
            blocks = [b.iloc[:5]] + blocks + [b.iloc[5:]]
        elif order == "cells_unsorted":
            q = np.random.default_rng(seed + 1).permutation(len(blocks[0]))
            blocks = [b.iloc[q] for b in blocks]
        df = pd.concat(blocks).reset_index(drop=True)
    if nan_locus:                   # one locus missing in one cell: dropped for every cell
        c0 = df.cell_id.iloc[0]
        df.loc[(df.cell_id == c0) & (df.chr == "2") & (df.start == 1), "reads"] = np.nan
    if shared:
        # one Python object per distinct label (as np.repeat-built or CSV-parsed tables hold
        # them): the per-cell block layout is then recognised from object identity
        for c in ("cell_id", "chr", "library_id", "clone_id", "note"):
            canon = {}
            df[c] = pd.Series([canon.setdefault(v, v) for v in df[c].tolist()], dtype=object)
    return df


def _ref_sort(cn):
    cn = cn.copy()
    cn["chr"] = cn["chr"].astype(str).astype("category").cat.set_categories(CHR)
    return cn.sort_values(by=["cell_id", "chr", "start"])


def _ref_process(cn_s, cn_g1):
    """pert_model.py:133-191 in plain pandas (pivot_table / dropna / .T)."""
    cn_g1 = _ref_sort(cn_g1)
    cn_s = _ref_sort(cn_s)
    cn_g1 = cn_g1[cn_g1["reads"].notna()]
    cn_s = cn_s[cn_s["reads"].notna()]
    piv = lambda df, col: df.pivot_table(index="cell_id", columns=["chr", "start"], values=col,
                                         observed=False).dropna(axis=1).T
    g_r, g_s, s_r, s_s = piv(cn_g1, "reads"), piv(cn_g1, "state"), piv(cn_s, "reads"), piv(cn_s, "state")
    libs_s = cn_s[["cell_id", "library_id"]].drop_duplicates()
    libs_g = cn_g1[["cell_id", "library_id"]].drop_duplicates()
    ids = list(pd.concat([libs_s, libs_g])["library_id"].unique())
    lut = {v: i for i, v in enumerate(ids)}
    gam = cn_s[["chr", "start", "gc"]].drop_duplicates().dropna()
    return dict(cn_s=cn_s, cn_g1=cn_g1, g_r=g_r, g_s=g_s, s_r=s_r, s_s=s_s,
                libs_s=libs_s["library_id"].map(lut).to_numpy(), libs_g=libs_g["library_id"].map(lut).to_numpy(),
                ids=ids, gc=gam["gc"].to_numpy(np.float32))


@pytest.mark.parametrize("shared", [False, True])
@pytest.mark.parametrize("order", ["shuffled", "cells", "cells_split", "cells_unsorted"])
@pytest.mark.parametrize("nan_locus", [False, True])
def test_process_input_data_matches_pandas(nan_locus, order, shared):
    s = _table(9, "s", seed=1, nan_locus=nan_locus, order=order, shared=shared)
    g = _table(6, "g", seed=2, n_libs=3, nan_locus=nan_locus, order=order, shared=shared)
    ref = _ref_process(s, g)
    blocks, layouts = [], []
    real, real_lay = prep._cell_blocks, prep._block_layout
    prep._cell_blocks = lambda *a: blocks.append(real(*a)) or blocks[-1]
    prep._block_layout = lambda *a: layouts.append(real_lay(*a)) or layouts[-1]
    try:
        cn_s, cn_g1, inp = prep.process_input_data(s, g)
    finally:
        prep._cell_blocks, prep._block_layout = real, real_lay
    # whole per-cell blocks: recognised from the labels' object identity (the block path,
    # no per-row hashing) where the labels are shared objects and no read is missing, else
    # by the per-cell block permutation of the general path
    per_cell = order in ("cells", "cells_unsorted")
    fast = per_cell and shared and not nan_locus
    assert [x is not None for x in layouts] == [fast] * 2
    assert [b is not None for b in blocks] == ([] if fast else [per_cell] * 2)
    if fast:
        assert isinstance(inp.keys_s, prep.RegularKeys) and isinstance(inp.keys_g, prep.RegularKeys)
    # sorted long tables: same rows in the same order, same columns and dtypes
    pd.testing.assert_frame_equal(cn_s, ref["cn_s"])
    pd.testing.assert_frame_equal(cn_g1, ref["cn_g1"])
    np.testing.assert_array_equal(inp.cells_s, ref["s_r"].columns.to_numpy())
    np.testing.assert_array_equal(inp.cells_g, ref["g_r"].columns.to_numpy())
    np.testing.assert_array_equal(inp.loci_chr.astype(str), ref["s_r"].index.get_level_values(0).astype(str))
    np.testing.assert_array_equal(inp.loci_start, ref["s_r"].index.get_level_values(1))
    t32 = lambda df: df.to_numpy().astype(np.int64).astype(np.float32)
    np.testing.assert_array_equal(inp.reads_s, t32(ref["s_r"]))
    np.testing.assert_array_equal(inp.reads_g, t32(ref["g_r"]))
    np.testing.assert_array_equal(inp.states_g, t32(ref["g_s"]))
    if not nan_locus:
        np.testing.assert_array_equal(inp.states_s, t32(ref["s_s"]))
        np.testing.assert_array_equal(inp.gc, ref["gc"])
    np.testing.assert_array_equal(inp.libs_s, ref["libs_s"])
    np.testing.assert_array_equal(inp.libs_g, ref["libs_g"])
    assert inp.library_ids == ref["ids"]


def test_pivot_averages_duplicates_and_drops_nan_keys():
    df = pd.DataFrame(dict(cell_id=["b", "a", "a", "b", "a", None], chr=["1", "1", "1", "2", "Z", "1"],
                           start=[1, 1, 1, 1, 1, 1], v=[1.0, 2.0, 4.0, 5.0, 9.0, 7.0]))
    p = prep.pivot_cells_by_loci(df, "v", "cell_id", "chr", "start")
    assert list(p.cells) == ["a", "b"]
    assert list(p.loci_chr) == ["1", "2"]
    np.testing.assert_array_equal(p.values, [[3.0, 1.0], [np.nan, 5.0]])


@pytest.mark.parametrize("col,with_keys", [("copy", False), ("state", False), ("copy", True), ("state", True)])
def test_consensus_clone_profiles_matches_pandas(col, with_keys):
    """Float values (median by sort) and integer states (median by histogram); on the raw
    table, or on the sorted table with its integer keys (the run_pert_model path)."""
    from scipy.stats import mode
    g = _table(10, "g", seed=3)
    g.loc[g.cell_id == g.cell_id.iloc[0], "state"] = 7            # an off-ploidy cell
    g.loc[g.cell_id == g.cell_id.iloc[1], "state"] = 3            # an even state count: half-way medians
    if with_keys:
        gs, keys = prep._sorted_table(g, "cell_id", "chr", "start")
        got = prep.consensus_clone_profiles(gs, col, keys=keys)
    else:
        got = prep.consensus_clone_profiles(g, col)
    # compute_consensus_clone_profiles.py:42-88 restated
    cn = g[g["clone_id"] != "None"].copy()
    pl = {c: mode(grp["state"], keepdims=False)[0] for c, grp in cn.groupby("cell_id")}
    cn["ploidy"] = cn["cell_id"].map(pl)
    pieces = []
    for _, grp in cn.groupby("clone_id"):
        keep = grp.groupby("ploidy").size().idxmax()
        pieces.append(grp[grp["ploidy"] == keep])
    cn = pd.concat(pieces, ignore_index=True)
    ref = cn.pivot_table(index=["chr", "start"], columns="clone_id", values=col, aggfunc="median")
    ref.index = pd.MultiIndex.from_arrays([ref.index.get_level_values(0).astype(str), ref.index.get_level_values(1)])
    got.index = pd.MultiIndex.from_arrays([got.index.get_level_values(0).astype(str), got.index.get_level_values(1)])
    got = got.loc[ref.index, ref.columns]
    np.testing.assert_allclose(got.to_numpy(), ref.to_numpy())


def test_clone_prior_matches_dense_reference():
    s = _table(8, "s", seed=4)
    g = _table(6, "g", seed=5)
    cn_s, cn_g1, inp = prep.process_input_data(s, g)
    prof = prep.consensus_clone_profiles(cn_g1, "state")
    eta = prep.build_clone_cn_prior(cn_s, inp.cells_s, inp.loci_chr, inp.loci_start, prof, 1e6, 13)
    dense = eta.dense()
    # pert_model.py:285-296: eta[:, n, clone_profile[l]] = weight, ones elsewhere
    idx = pd.MultiIndex.from_arrays([prof.index.get_level_values(0).astype(str), prof.index.get_level_values(1)])
    li = idx.get_indexer(pd.MultiIndex.from_arrays([inp.loci_chr.astype(str), inp.loci_start]))
    for n, cell in enumerate(inp.cells_s):
        clone = cn_s.loc[cn_s.cell_id == cell, "clone_id"].values[0]
        st = prof[clone].to_numpy()[li].astype(np.int64)
        want = np.ones((len(li), 13), np.float32)
        want[np.arange(len(li)), st] = 1e6
        np.testing.assert_array_equal(dense[:, n], want)


@pytest.mark.parametrize("bad", [13.0, -1.0, 65536.0 + 2.0])
def test_clone_prior_refuses_out_of_range_states(bad):
    """A clone profile state outside [0, P) is refused (build_cn_prior's range check), also one
    that narrowing to the uint16 codes would wrap into range."""
    s = _table(8, "s", seed=4)
    g = _table(6, "g", seed=5)
    cn_s, cn_g1, inp = prep.process_input_data(s, g)
    prof = prep.consensus_clone_profiles(cn_g1, "state").copy()
    prof.iloc[3, 0] = bad
    with pytest.raises(ValueError):
        prep.build_clone_cn_prior(cn_s, inp.cells_s, inp.loci_chr, inp.loci_start, prof, 1e6, 13)


def test_column_median_equals_numpy():
    """prep._column_median (threaded locus tiles) is np.median(vals[rows], axis=0)."""
    rng = np.random.default_rng(6)
    for n, L in [(1, 7), (300, 600), (65, 257)]:
        for v in (rng.integers(0, 9, (n, L)).astype(np.float64), rng.normal(size=(n, L))):
            rows = np.sort(rng.choice(n, size=max(1, n // 2), replace=False))
            np.testing.assert_array_equal(prep._column_median(v, rows), np.median(v[rows], axis=0))


def test_consensus_matches_reference_golden():
    """prep.consensus_clone_profiles against the reference's own compute_consensus_clone_profiles
    output (tests/golden/make_reference_golden.py; cn_state_col=None path, unsorted rows,
    missing rows, a 'None' clone)."""
    import os
    import pandas as pd
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "consensus_reference.npz"))
    df = pd.DataFrame({"cell_id": g["cell_id"].astype(object), "chr": g["chr"].astype(object), "start": g["start"],
                       "clone_id": g["clone_id"].astype(object), "copy": g["copy"]})
    got = prep.consensus_clone_profiles(df, "copy", clone_col="clone_id", cell_col="cell_id", chr_col="chr",
                                        start_col="start", cn_state_col=None)
    assert list(np.asarray(got.columns).astype(str)) == list(g["prof_clones"])
    assert list(np.asarray(got.index.get_level_values(0)).astype(str)) == list(g["prof_chr"])
    assert (np.asarray(got.index.get_level_values(1)) == g["prof_start"]).all()
    np.testing.assert_array_equal(got.to_numpy(np.float64), g["prof_values"])


@pytest.mark.parametrize("complete", [True, False])
def test_cell_in_two_libraries_is_refused(complete):
    """get_libraries_tensor (:206-225) asserts one library per cell; both the regular-table
    path and the general one raise."""
    s = _table(6, "s", seed=4)
    g = _table(5, "g", seed=5)
    c0 = s.cell_id.iloc[0]
    rows = s.index[s.cell_id == c0]
    s.loc[rows[:3], "library_id"] = "L_other"
    if not complete:                                   # a duplicated row: not a regular table
        s = pd.concat([s, s.iloc[[len(s) - 1]]], ignore_index=True)
    with pytest.raises(ValueError, match="more than one"):
        prep.process_input_data(s, g)


def test_block_path_keys_serve_every_consumer():
    """The block path's RegularKeys give the consumers of the keys (consensus profiles, the
    clone prior's first rows, the general pivot) what the general path's TableKeys give."""
    s = _table(9, "s", seed=4, order="cells_unsorted", shared=True)
    g = _table(8, "g", seed=5, n_libs=3, order="cells_unsorted", shared=True)
    cn_s, cn_g1, inp = prep.process_input_data(s, g)
    assert isinstance(inp.keys_g, prep.RegularKeys)
    kg = prep.TableKeys(cn_g1, "cell_id", "chr", "start")
    np.testing.assert_array_equal(inp.keys_g.cell_code, kg.cell_code)
    np.testing.assert_array_equal(inp.keys_g.locus_code, kg.locus_code)
    np.testing.assert_array_equal(inp.keys_g.cells, kg.cells)
    np.testing.assert_array_equal(inp.keys_g.loci_start, kg.loci_start)
    assert inp.keys_g.regular == kg.regular
    for col in ("state", "copy"):
        pd.testing.assert_frame_equal(prep.consensus_clone_profiles(cn_g1, col, keys=inp.keys_g),
                                      prep.consensus_clone_profiles(cn_g1, col, keys=kg))
    np.testing.assert_array_equal(prep.first_clone(cn_s, inp.cells_s, keys=inp.keys_s),
                                  prep.first_clone(cn_s, inp.cells_s))
    p1 = prep.pivot_cells_by_loci(cn_g1, "reads", "cell_id", "chr", "start", inp.keys_g)
    p2 = prep.pivot_cells_by_loci(cn_g1, "reads", "cell_id", "chr", "start")
    np.testing.assert_array_equal(p1.values, p2.values)


def test_scrt_consensus_block_path_equals_general_path():
    """infer_scRT.consensus_profiles (a per-cell block table sorted into a temporary copy with
    RegularKeys) returns the general path's profiles exactly: index, columns, dtypes, values."""
    from scdna_replication_tools_amd.infer_scRT import consensus_profiles
    from scdna_replication_tools_amd.simulator import simulate, to_long_form
    sim = simulate(n_s=4, n_g=90, n_bins=400, num_reads=400 * 183, seed=4, n_clones=3)
    _, df_g = to_long_form(sim, n_libs=1, copy_from="reads")
    assert prep._block_layout(df_g, "cell_id", "chr", "start", None) is not None
    for col in ("copy", "state"):
        a = prep.consensus_clone_profiles(df_g, col, clone_col="clone_id", cn_state_col="state")
        b = consensus_profiles(df_g, col, clone_col="clone_id", cn_state_col="state")
        pd.testing.assert_frame_equal(a, b)


@pytest.mark.parametrize("kind", ["int", "categorical"])
def test_scrt_consensus_block_path_keeps_caller_chr_labels(kind):
    """Integer chromosome labels stay integers in numeric order, a categorical chr column keeps
    its own categories -- as the general path (pivot_table) returns them -- over several
    chromosomes (the block path sorts a copy whose labels are CHR_ORDER strings)."""
    from scdna_replication_tools_amd.infer_scRT import consensus_profiles
    from scdna_replication_tools_amd.simulator import simulate, to_long_form
    sim = simulate(n_s=2, n_g=12, n_bins=5451, num_reads=5451 * 50, seed=5, n_clones=2)
    _, df_g = to_long_form(sim, n_libs=1, copy_from="reads")
    df_g = df_g[~df_g["chr"].astype(str).isin(["X", "Y"])].reset_index(drop=True)   # integer-labelled autosomes
    assert df_g["chr"].nunique() > 10
    if kind == "int":
        df_g["chr"] = df_g["chr"].astype(str).astype(np.int64)
    else:
        cats = sorted(df_g["chr"].astype(str).unique()) + ["MT"]
        df_g["chr"] = pd.Categorical(df_g["chr"].astype(str), categories=cats)
    assert prep._block_layout(df_g, "cell_id", "chr", "start", None) is not None
    a = prep.consensus_clone_profiles(df_g, "copy", clone_col="clone_id", cn_state_col="state")
    b = consensus_profiles(df_g, "copy", clone_col="clone_id", cn_state_col="state")
    pd.testing.assert_frame_equal(a, b)


def test_pivot_any_block_path_equals_general_pivot():
    from scdna_replication_tools_amd.simulator import simulate, to_long_form
    sim = simulate(n_s=4, n_g=30, n_bins=300, num_reads=300 * 183, seed=6)
    _, df_g = to_long_form(sim, n_libs=1, copy_from="reads")
    for col in ("copy", "reads", "state"):
        a = prep.pivot_cells_by_loci(df_g, col, "cell_id", "chr", "start")
        b = prep.pivot_any(df_g, col, "cell_id", "chr", "start")
        assert list(a.cells) == list(b.cells) and list(a.loci_chr) == list(b.loci_chr)
        np.testing.assert_array_equal(a.loci_start, b.loci_start)
        np.testing.assert_array_equal(np.asarray(a.values, np.float64), np.asarray(b.values, np.float64))


@pytest.mark.parametrize("kind", ["int", "bigint", "float"])
def test_block_pivot_tiles_equal_whole_transpose(kind):
    """_block_pivot's threaded cell tiles (gather + transpose + cast per 64 cells) equal the
    whole-matrix gather and transpose, across several tiles and a ragged last one."""
    rng = np.random.default_rng(3)
    B, L = 300, 37
    v = {"int": rng.integers(0, 90, B * L), "bigint": rng.integers(0, 1 << 40, B * L),
         "float": rng.normal(size=B * L)}[kind]
    for bp, q in [(np.arange(B), np.arange(L)), (rng.permutation(B), rng.permutation(L))]:
        got = prep._block_pivot(v, B, L, bp, q)
        want = v.reshape(B, L)[bp][:, q].T
        assert got.dtype == (np.float32 if kind == "int" else np.float64)
        np.testing.assert_array_equal(got, want.astype(got.dtype))


@pytest.mark.parametrize("shape", [(7, 1), (37, 300), (5, 64), (3, 65), (0, 5), (5, 0)])
def test_transpose_cast_equals_numpy(shape):
    """prep.transpose_cast (threaded cell tiles; package_s_output's (cell, locus) columns) is
    np.ascontiguousarray(a.T).astype(dtype), also for a non-contiguous view."""
    a = np.random.default_rng(5).integers(0, 13, shape).astype(np.uint8)
    for dt in (np.int64, np.float32):
        got = prep.transpose_cast(a, dt)
        assert got.dtype == dt
        np.testing.assert_array_equal(got, np.ascontiguousarray(a.T).astype(dt))
    v = a[:, 1:]
    np.testing.assert_array_equal(prep.transpose_cast(v, np.int64), v.T.astype(np.int64))


def test_row_state_counts_equals_bincount():
    """prep._row_state_counts (threaded row tiles) counts each row's states like one bincount."""
    rng = np.random.default_rng(8)
    for B, L, V in [(1, 5, 3), (300, 41, 7), (257, 3, 13)]:
        st = rng.integers(0, V, (B, L))
        want = np.stack([np.bincount(r, minlength=V) for r in st])
        np.testing.assert_array_equal(prep._row_state_counts(st, V), want)
        np.testing.assert_array_equal(prep._row_state_counts(st.astype(np.float64), V), want)


@pytest.mark.parametrize("kind", [1, 2, 3])
@pytest.mark.parametrize("method", ["sampled", "median"])
def test_init_params_of_a_cell_range_equal_the_whole_fits(kind, method):
    """init_params(cells=...) -- one rank's shard of a sharded fit -- gives exactly the whole
    fit's initial values of those cells (the generator still draws for every cell), with
    t_init / ploidy given for the rank's cells only; the shared sites are the whole fit's."""
    from scdna_replication_tools_amd.init import init_params
    rng = np.random.default_rng(3)
    L, N, n_libs = 40, 37, 2
    reads = rng.poisson(100, (L, N)).astype(np.float32)
    libs = rng.integers(0, n_libs, N)
    ploidy = rng.uniform(1.5, 3.0, N)
    t_init = rng.uniform(0.05, 0.95, N)
    bm = rng.normal(size=(n_libs, 5))
    kw = dict(beta_means=bm, seed=7, method=method)
    whole = init_params(kind, reads, libs, n_libs, 13, 4, ploidy=ploidy, t_init=t_init, **kw)
    for sl in (slice(0, 19), slice(19, N), slice(5, 6)):
        part = init_params(kind, reads, libs, n_libs, 13, 4, ploidy=ploidy[sl], t_init=t_init[sl], cells=sl, **kw)
        assert set(part) == set(whole)
        for k, v in whole.items():
            want = v[sl] if k in ("expose_tau", "expose_u", "expose_betas") else v
            np.testing.assert_array_equal(part[k], want, err_msg=k)


def test_clone_prior_of_a_cell_range_equals_the_whole_prior_sliced():
    """build_clone_cn_prior(cell_range=...) -- one rank's code book -- equals the whole code
    book's columns of those cells; an out-of-range clone state raises on every rank alike."""
    from scdna_replication_tools_amd.simulator import simulate, to_long_form
    from scdna_replication_tools_amd.pert_model import pert_infer_scRT
    sim = simulate(n_s=23, n_g=30, n_bins=300, num_reads=300 * 183, seed=8, n_clones=3)
    s, g = to_long_form(sim, n_libs=1)
    m = pert_infer_scRT(s, g, input_col='reads', clone_col='clone_id', cn_prior_method='g1_clones', device="cpu")
    inp = m._prepare()
    profiles = prep.consensus_clone_profiles(m.cn_g1, m.cn_state_col, keys=inp.keys_g)
    whole = m._build_etas(inp, profiles)
    for sl in (slice(0, 12), slice(12, 23)):
        part = m._build_etas(inp, profiles, cells=sl)
        np.testing.assert_array_equal(part.codes, whole.codes[:, sl])
        np.testing.assert_array_equal(part.table, whole.table)
        np.testing.assert_array_equal(part.ploidy(), whole.ploidy()[sl])
    for method in ("hmmcopy", "diploid", "uniform", "g1_composite"):
        m.cn_prior_method = method
        w = m._build_etas(inp, profiles)
        p = m._build_etas(inp, profiles, cells=slice(3, 17))
        np.testing.assert_array_equal(p.dense(), w.dense()[:, 3:17], err_msg=method)


def test_scrt_consensus_block_path_any_block_and_locus_order():
    """The consensus from the table's blocks as they lie (cells in any order, every block's loci
    in one shared but unsorted order, a clone 'None' cell): the general path's profiles exactly."""
    from scdna_replication_tools_amd.infer_scRT import consensus_profiles
    from scdna_replication_tools_amd.simulator import simulate, to_long_form
    sim = simulate(n_s=4, n_g=60, n_bins=400, num_reads=400 * 183, seed=9, n_clones=3)
    _, df_g = to_long_form(sim, n_libs=1, copy_from="reads")
    B = df_g["cell_id"].nunique()
    L = len(df_g) // B
    rng = np.random.default_rng(2)
    cell_perm, locus_perm = rng.permutation(B), rng.permutation(L)
    order = (cell_perm[:, None] * L + locus_perm[None, :]).reshape(-1)
    df = df_g.iloc[order].reset_index(drop=True)
    first = df["cell_id"].to_numpy()[0]
    df.loc[df["cell_id"] == first, "clone_id"] = "None"
    assert prep._block_layout(df, "cell_id", "chr", "start", None) is not None
    for col in ("copy", "state"):
        a = prep.consensus_clone_profiles(df, col, clone_col="clone_id", cn_state_col="state")
        b = consensus_profiles(df, col, clone_col="clone_id", cn_state_col="state")
        pd.testing.assert_frame_equal(a, b)


def test_process_input_data_deferred_sorted_tables_equal_eager():
    """defer_sorted (run_pert_model): the sorted copies of per-cell-block tables built on a
    background thread -- the same inputs, library index and gc as the eager path, the same
    sorted tables once resolved, and the per-cell labels (first_clone, libraries) and the
    consensus read from the source blocks equal to those of the sorted copies."""
    from scdna_replication_tools_amd.simulator import simulate, to_long_form
    sim = simulate(n_s=20, n_g=30, n_bins=300, num_reads=300 * 183, seed=12, n_clones=3)
    df_s, df_g = to_long_form(sim, n_libs=2)
    rng = np.random.default_rng(3)
    B = df_s["cell_id"].nunique()
    L = len(df_s) // B
    order = (rng.permutation(B)[:, None] * L + rng.permutation(L)[None, :]).reshape(-1)
    df_s = df_s.iloc[order].reset_index(drop=True)                  # blocks and loci in another order
    seen = {}
    s1, g1, a = prep.process_input_data(df_s, df_g)
    s2, g2, b = prep.process_input_data(df_s, df_g, defer_sorted=True,
                                        on_g1_sorted=lambda t, k: seen.setdefault("g", (t, k)))
    assert isinstance(s2, prep.DeferredTable) and isinstance(seen["g"][0], prep.DeferredTable)
    for f in ("reads_s", "reads_g", "states_s", "states_g", "gc", "libs_s", "libs_g", "cells_s", "cells_g",
              "loci_chr", "loci_start"):
        np.testing.assert_array_equal(getattr(a, f), getattr(b, f), err_msg=f)
    assert a.library_ids == b.library_ids
    for name, (x, y) in {"clone_id": (s1, s2), "library_id": (g1, g2)}.items():
        rows = np.arange(len(x))[::7]
        np.testing.assert_array_equal(x[name].to_numpy()[rows], y.column_at(name, rows))
    np.testing.assert_array_equal(prep.first_clone(s1, a.cells_s, keys=a.keys_s),
                                  prep.first_clone(s2, b.cells_s, keys=b.keys_s))
    pa = prep.consensus_clone_profiles(g1, "state", keys=a.keys_g)
    pb = prep.consensus_clone_profiles(seen["g"][0], "state", keys=seen["g"][1])
    pd.testing.assert_frame_equal(pa, pb)
    pd.testing.assert_frame_equal(s1, prep.resolved(s2))
    pd.testing.assert_frame_equal(g1, prep.resolved(g2))


@pytest.mark.parametrize("kind", [1, 2, 3])
def test_init_params_median_of_quantiles_equals_quantile_of_median(kind):
    """init._median15 takes one quantile per site (median first): the initial values equal the
    median of the 15 quantiles, bit for bit, for every site of the three fits."""
    from scdna_replication_tools_amd import init as init_mod

    def median15_literal(rng, ppf, shape):
        u = rng.uniform(1e-12, 1 - 1e-12, size=(15,) + tuple(shape))
        return np.median(ppf(u), axis=0)
    rng = np.random.default_rng(4)
    N, L = 3000, 400
    reads = rng.poisson(50, size=(L, N)).astype(np.float32)
    libs = rng.integers(0, 2, N)
    kw = dict(ploidy=rng.uniform(1.5, 4, N), t_init=rng.uniform(0.05, 0.95, N),
              beta_means=rng.normal(size=(2, 5))) if kind != 1 else {}
    a = init_mod.init_params(kind, reads, libs, 2, 13, 4, seed=7, **kw)
    orig = init_mod._median15
    init_mod._median15 = median15_literal
    try:
        b = init_mod.init_params(kind, reads, libs, 2, 13, 4, seed=7, **kw)
    finally:
        init_mod._median15 = orig
    assert a.keys() == b.keys()
    for k in a:
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)
