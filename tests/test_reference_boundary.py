"""The drop-in surface (CPU): the reference's import paths, constructor, public helper
methods and output packaging.

``package_s_output`` is checked against a literal restatement of the reference's
melt + merge code (pert_model.py:466-538); the helper methods against literal
restatements of their reference loops (pert_model.py:206-296).  The prior builders of
the correlation-matched methods are in tests/test_priors.py.
"""
import inspect
import os

import numpy as np
import pandas as pd
import pytest
import torch

from tests.test_prep import CHR, _ref_process, _table


def _model(seed=6, n_s=8, n_g=6, drop_locus=False):
    from scdna_replication_tools_amd.pert_model import pert_infer_scRT
    s = _table(n_s, "s", seed=seed, nan_locus=drop_locus)
    g = _table(n_g, "g", seed=seed + 1, nan_locus=drop_locus)
    return pert_infer_scRT(s, g, cn_prior_method='g1_clones', device='cpu'), s, g


def _ref_package(cn_s, trace, cn_s_reads_df, lambda_fit, losses_g, losses_s):
    """pert_model.py:466-538, restated line by line (reference's pandas calls)."""
    cn_s = cn_s.copy()
    u, rho, a, tau = (trace[k] for k in ("expose_u", "expose_rho", "expose_a", "expose_tau"))
    model_cn_df = pd.DataFrame(trace["cn"], index=cn_s_reads_df.index, columns=cn_s_reads_df.columns)
    model_rep_df = pd.DataFrame(trace["rep"], index=cn_s_reads_df.index, columns=cn_s_reads_df.columns)
    model_cn_df = model_cn_df.melt(ignore_index=False, value_name='model_cn_state').reset_index()
    model_rep_df = model_rep_df.melt(ignore_index=False, value_name='model_rep_state').reset_index()
    out = pd.merge(cn_s, model_cn_df)
    out = pd.merge(out, model_rep_df)
    taus = pd.DataFrame(tau, index=cn_s_reads_df.columns, columns=['model_tau']).reset_index()
    us = pd.DataFrame(u, index=cn_s_reads_df.columns, columns=['model_u']).reset_index()
    rhos = pd.DataFrame(rho, index=cn_s_reads_df.index, columns=['model_rho']).reset_index()
    out = pd.merge(out, taus)
    out = pd.merge(out, us)
    out = pd.merge(out, rhos)
    supp = pd.concat([
        pd.DataFrame({'param': ['model_lambda'], 'level': ['all'], 'value': [lambda_fit[0]]}),
        pd.DataFrame({'param': ['model_a'], 'level': ['all'], 'value': [a[0]]}),
        pd.DataFrame({'param': ['loss_g'] * len(losses_g), 'level': np.arange(len(losses_g)), 'value': losses_g}),
        pd.DataFrame({'param': ['loss_s'] * len(losses_s), 'level': np.arange(len(losses_s)), 'value': losses_s}),
    ], ignore_index=True)
    return out, supp


@pytest.mark.parametrize("drop_locus", [False, True])
def test_package_s_output_matches_reference_melt_merge(drop_locus):
    """Rows, row order, columns and dtypes of the reference's inner merges, on a table with
    shuffled rows, several chromosomes and (drop_locus) a locus missing in one cell, which
    the pivot drops for every cell and the merges drop from the output."""
    from scdna_replication_tools_amd.pert_model import MapTrace
    m, s, g = _model(drop_locus=drop_locus)
    tup = m.process_input_data()
    cn_s_reads_df = tup[2]
    L, N = cn_s_reads_df.shape
    rng = np.random.default_rng(0)
    tr = {"cn": rng.integers(0, 13, (L, N)), "rep": rng.integers(0, 2, (L, N)).astype(np.float32),
          "expose_tau": rng.uniform(size=N).astype(np.float32), "expose_u": rng.uniform(50, 90, N).astype(np.float32),
          "expose_rho": rng.uniform(size=(L, 1)).astype(np.float32), "expose_a": np.array([7.5], np.float32)}
    lam = np.array([0.71], np.float32)
    lg, ls = [3.0, 2.0, 1.5], [9.0, 8.5]
    got, gsupp = m.package_s_output(m.cn_s, MapTrace(**{k: torch.as_tensor(v) for k, v in tr.items()}),
                                    cn_s_reads_df, torch.as_tensor(lam), lg, ls)
    ref, rsupp = _ref_package(m.cn_s, tr, cn_s_reads_df, lam, lg, ls)
    pd.testing.assert_frame_equal(got, ref)
    pd.testing.assert_frame_equal(gsupp, rsupp)
    if drop_locus:
        assert len(got) < len(m.cn_s)
    # the fast path of run_pert_model (integer keys of the sorted table, no frame) agrees
    from scdna_replication_tools_amd.pert_model import PivotAxes
    inp = m._prepare()
    fast, _ = m.package_s_output(m.cn_s, MapTrace(**tr), PivotAxes(inp.loci_chr, inp.loci_start, inp.cells_s,
                                                                  keys=inp.keys_s), lam, lg, ls)
    pd.testing.assert_frame_equal(fast, ref)


def test_process_input_data_returns_reference_tuple():
    m, s, g = _model(seed=3)
    out = m.process_input_data()
    assert len(out) == 12
    g_r_df, g_s_df, s_r_df, s_s_df, g_r, g_s, s_r, s_s, gammas, rt_prior, libs_g, libs_s = out
    ref = _ref_process(s, g)
    t32 = lambda df: df.to_numpy().astype(np.int64).astype(np.float32)
    np.testing.assert_array_equal(s_r.numpy(), t32(ref["s_r"]))
    np.testing.assert_array_equal(g_s.numpy(), t32(ref["g_s"]))
    assert list(s_r_df.columns) == list(ref["s_r"].columns)
    assert list(s_r_df.index.get_level_values(1)) == list(ref["s_r"].index.get_level_values(1))
    assert s_r_df.columns.name == "cell_id" and list(s_r_df.index.names) == ["chr", "start"]
    np.testing.assert_array_equal(gammas.numpy(), ref["gc"])
    assert rt_prior is None                       # the test tables carry no mcf7rt column
    assert s_r.dtype == torch.float32 and libs_s.dtype == torch.int64
    np.testing.assert_array_equal(libs_s.numpy(), ref["libs_s"])
    assert m.L == len(ref["ids"])


def test_reference_helper_methods():
    m, s, g = _model(seed=4)
    cn_s, cn_g1 = m.sort_by_cell_and_loci(s.copy()), m.sort_by_cell_and_loci(g.copy())
    # get_libraries_tensor (pert_model.py:206-225): replace() loop over first-appearance ids
    ls_, lg_ = m.get_libraries_tensor(cn_s, cn_g1)
    a = cn_s[["cell_id", "library_id"]].drop_duplicates()
    b = cn_g1[["cell_id", "library_id"]].drop_duplicates()
    ids = pd.concat([a, b])["library_id"].unique()
    with pd.option_context("future.no_silent_downcasting", True):
        for i, lib in enumerate(ids):
            a = a.replace({"library_id": {lib: i}})
            b = b.replace({"library_id": {lib: i}})
    np.testing.assert_array_equal(ls_.numpy(), a["library_id"].to_numpy(np.int64))
    np.testing.assert_array_equal(lg_.numpy(), b["library_id"].to_numpy(np.int64))
    assert m.L == len(ids)
    # make_g1_g2_training_data (:228-251)
    st = torch.randint(0, 5, (9, 4)).float()
    rd = torch.rand(9, 4)
    lb = torch.tensor([0, 1, 0, 1])
    s2, r2, l2, rep2 = m.make_g1_g2_training_data(st, rd, lb)
    assert s2.shape == (9, 8) and (rep2[:, :4] == 0).all() and (rep2[:, 4:] == 1).all()
    assert torch.equal(l2, torch.cat([lb, lb])) and torch.equal(r2[:, 4:], rd)
    # build_trans_mat (:260-269): the per-cell / per-locus loop
    cn = torch.randint(0, 13, (30, 5))
    want = torch.eye(13, 13) + 1
    for i in range(5):
        for j in range(1, 30):
            want[int(cn[j - 1, i]), int(cn[j, i])] += 1
    assert torch.equal(m.build_trans_mat(cn), want)
    # build_cn_prior (:272-282): the per-element loop
    st = torch.randint(0, 13, (6, 7)).float()
    want = torch.ones(6, 7, 13)
    for i in range(6):
        for n in range(7):
            want[i, n, int(st[i, n].numpy())] = 1e6
    assert torch.equal(m.build_cn_prior(st), want)
    assert torch.equal(m.build_cn_prior(st, weight=5.0)[0, 0], torch.where(want[0, 0] > 1, 5.0, 1.0))
    # make_gc_features (:460-463)
    x = torch.tensor([0.3, 0.5])
    f = m.make_gc_features(x)
    assert f.shape == (2, 5) and torch.allclose(f[:, 0], x ** 4) and torch.equal(f[:, -1], torch.ones(2))
    # convert_rt_prior_units (:254-257)
    r = torch.tensor([[1.0], [4.0], [2.0]])
    assert torch.equal(m.convert_rt_prior_units(r), r / 4.0)


def test_clone_prior_method_matches_reference_loop():
    """build_clone_cn_prior(cn, cn_df, cn_tensor, clone_cn_profiles) (pert_model.py:285-296)."""
    m, s, g = _model(seed=8)
    tup = m.process_input_data()
    cn_s_reads_df, cn_s_states = tup[2], tup[7]
    from scdna_replication_tools_amd.prep import consensus_clone_profiles
    prof = consensus_clone_profiles(m.cn_g1, "state")
    got = m.build_clone_cn_prior(m.cn_s, cn_s_reads_df, cn_s_states, prof)
    inp = torch.zeros(cn_s_states.shape)
    for i, cell_id in enumerate(cn_s_reads_df.columns):
        cell_clone = m.cn_s.loc[m.cn_s["cell_id"] == cell_id]["clone_id"].values[0]
        inp[:, i] = torch.tensor(prof[cell_clone].values).to(torch.int64).to(torch.float32)
    assert torch.equal(got, m.build_cn_prior(inp))


def test_import_paths_and_signatures_match_reference():
    """notebooks: `from scdna_replication_tools.infer_scRT import scRT` (inference_tutorial
    cell 1); the constructors keep the reference's parameters, order and defaults
    (infer_scRT.py:26-31, pert_model.py:37-43)."""
    from scdna_replication_tools.infer_scRT import scRT
    from scdna_replication_tools.pert_model import pert_infer_scRT
    from scdna_replication_tools.compute_consensus_clone_profiles import compute_consensus_clone_profiles  # noqa
    from scdna_replication_tools.predict_cycle_phase import predict_cycle_phase  # noqa
    from scdna_replication_tools.cncluster import kmeans_cluster  # noqa
    from scdna_replication_tools.assign_s_to_clones import assign_s_to_clones  # noqa
    from scdna_replication_tools.normalize_by_cell import compute_cell_corrs  # noqa
    ref_pert = ["cn_s", "cn_g1", "input_col", "gc_col", "rt_prior_col", "clone_col", "cell_col", "library_col",
                "chr_col", "start_col", "cn_state_col", "assign_col", "rs_col", "frac_rt_col", "cn_prior_method",
                "cn_prior_weight", "learning_rate", "max_iter", "min_iter", "rel_tol", "max_iter_step1",
                "min_iter_step1", "max_iter_step3", "min_iter_step3", "cuda", "seed", "P", "K", "J", "upsilon",
                "run_step3"]
    sig = inspect.signature(pert_infer_scRT.__init__)
    names = [p for p in sig.parameters if p != "self"]
    assert names[:len(ref_pert)] == ref_pert
    d = {p: sig.parameters[p].default for p in ref_pert[2:]}
    assert d["cn_prior_method"] == "g1_composite" and d["max_iter"] == 2000 and d["min_iter"] == 100
    assert d["P"] == 13 and d["K"] == 4 and d["J"] == 5 and d["upsilon"] == 6 and d["rel_tol"] == 1e-6
    assert d["learning_rate"] == 0.05 and d["cn_prior_weight"] == 1e6 and d["run_step3"] is True
    ref_scrt = ["cn_s", "cn_g1", "input_col", "assign_col", "library_col", "ploidy_col", "cell_col", "cn_state_col",
                "chr_col", "start_col", "gc_col", "rv_col", "rs_col", "frac_rt_col", "clone_col", "rt_prior_col",
                "cn_prior_method", "col2", "col3", "col4", "col5", "max_iter", "min_iter", "max_iter_step1",
                "min_iter_step1", "max_iter_step3", "min_iter_step3", "cn_prior_weight", "learning_rate", "rel_tol",
                "cuda", "seed", "P", "K", "J", "upsilon", "run_step3"]
    sig = inspect.signature(scRT.__init__)
    assert [p for p in sig.parameters if p != "self"][:len(ref_scrt)] == ref_scrt
    assert sig.parameters["cn_prior_method"].default == "hmmcopy"
    for meth in ("process_input_data", "sort_by_cell_and_loci", "get_libraries_tensor", "make_g1_g2_training_data",
                 "convert_rt_prior_units", "build_trans_mat", "build_cn_prior", "build_clone_cn_prior",
                 "build_composite_cn_prior", "manhattan_binarization", "guess_times", "make_gc_features",
                 "package_s_output", "run_pert_model"):
        assert callable(getattr(pert_infer_scRT, meth)), meth
    ref_params = {"build_cn_prior": ["cn", "weight"], "build_clone_cn_prior": ["cn", "cn_df", "cn_tensor",
                                                                              "clone_cn_profiles"],
                  "build_composite_cn_prior": ["cn", "clone_cn_profiles", "weight"],
                  "guess_times": ["cn_s_reads", "etas"], "make_gc_features": ["x"],
                  "package_s_output": ["cn_s", "trace_s", "cn_s_reads_df", "lambda_fit", "losses_g", "losses_s"],
                  "manhattan_binarization": ["X", "MEAN_GAP_THRESH", "EARLY_S_SKEW_THRESH", "LATE_S_SKEW_THRESH"]}
    for meth, params in ref_params.items():
        assert [p for p in inspect.signature(getattr(pert_infer_scRT, meth)).parameters if p != "self"] == params
    assert inspect.signature(pert_infer_scRT.build_composite_cn_prior).parameters["weight"].default == 1e5


def test_reference_logging_and_per_step_lines(capsys):
    """Importing the drop-in pert_model configures root logging as the reference's import
    does (pert_model.py:25-33), and every fit logs 'step: i, loss: ...' on the root logger
    (:747, :805, :872); log_steps=False silences them."""
    import logging
    import subprocess
    import sys
    out = subprocess.run([sys.executable, "-c", "import logging, scdna_replication_tools.pert_model; "
                          "r = logging.getLogger(); print(r.level, len(r.handlers))"],
                         capture_output=True, text=True, check=True, cwd=os.path.dirname(os.path.dirname(__file__)))
    assert out.stdout.split() == ["10", "2"]                 # DEBUG; basicConfig's + the stdout handler
    root = logging.getLogger()
    m, s, g = _model(seed=2)

    class FakeShard:
        def run_svi(self, max_iter, min_iter, rel_tol):
            return [3.0, 2.5, 2.25], 1

    class Catch(logging.Handler):
        def __init__(self):
            super().__init__()
            self.msgs = []

        def emit(self, record):
            self.msgs.append(record.getMessage())

    h = Catch()
    root.addHandler(h)
    level = root.level
    root.setLevel(logging.INFO)
    try:
        m._svi(FakeShard(), 10, 1, "step2")
        assert h.msgs == ["step: 0, loss: 3.0", "step: 1, loss: 2.5", "step: 2, loss: 2.25"]
        assert "ELBO converged at iteration 2" in capsys.readouterr().out
        h.msgs.clear()
        m.log_steps = False
        m._svi(FakeShard(), 10, 1, "step2")
        assert h.msgs == []
    finally:
        root.removeHandler(h)
        root.setLevel(level)
