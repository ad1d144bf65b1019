"""KMeans + BIC clustering used when clone labels are absent (reference cncluster.py:50-120,
infer_scRT.py:129-138).  CPU: the BIC against a literal restatement of the reference's
per-cluster loop, and clone recovery on simulated polyclonal G1 cells for the batched
tensor backend and for sklearn's estimator.  The reference's fits are unseeded, so the
pin is behavioural (parity unpinned beyond that)."""
import numpy as np
import pandas as pd
import pytest

from scdna_replication_tools_amd import prep
from scdna_replication_tools_amd.cncluster import compute_bic, compute_bic_tensor, kmeans_cluster, kmeans_fit
from scdna_replication_tools_amd.simulator import simulate, to_long_form


def _bic_loop(centers, labels, X):
    """cncluster.py:62-77 as written (cdist per cluster, per-cluster sum)."""
    from scipy.spatial.distance import cdist
    n_clusters = centers.shape[0]
    cluster_sizes = np.bincount(labels)
    N, d = X.shape
    cl_var = (1.0 / (N - n_clusters) / d) * sum(
        [sum(cdist(X[np.where(labels == i)], [centers[i]], 'euclidean') ** 2) for i in range(n_clusters)])
    const_term = 0.5 * n_clusters * np.log(N) * (d + 1)
    return np.sum([cluster_sizes[i] * np.log(cluster_sizes[i]) - cluster_sizes[i] * np.log(N)
                   - ((cluster_sizes[i] * d) / 2) * np.log(2 * np.pi * cl_var) - ((cluster_sizes[i] - 1) * d / 2)
                   for i in range(n_clusters)]) - const_term


def test_bic_matches_reference_formula():
    """Both BIC implementations (host numpy, and the device-tensor one kmeans_cluster uses)
    against the reference's per-cluster loop."""
    import torch
    rng = np.random.default_rng(0)
    X = np.concatenate([rng.normal(m, 0.3, size=(40, 7)) for m in (0.0, 2.0, 5.0)])
    for k in (2, 3, 5):
        centers, labels, _ = kmeans_fit(X, k, n_init=4, device="cpu")
        ref = float(_bic_loop(centers, labels, X))
        assert np.isclose(compute_bic(centers, labels, X), ref, rtol=1e-10)
        got = compute_bic_tensor(torch.as_tensor(centers), torch.as_tensor(labels), torch.as_tensor(X))
        assert np.isclose(got, ref, rtol=1e-10)


def _g1_matrix(n=60, L=400, seed=3):
    sim = simulate(n_s=n, n_g=n, n_bins=L, num_reads=400 * L, seed=seed)
    _, df_g = to_long_form(sim, copy_from="reads")
    piv = prep.pivot_cells_by_loci(df_g, "copy", "cell_id", "chr", "start")
    mat = pd.DataFrame(piv.values, columns=piv.cells)
    truth = pd.Series(df_g.drop_duplicates("cell_id").set_index("cell_id")["clone_id"])
    return mat, truth


def _same_partition(a, b):
    t = pd.crosstab(np.asarray(a), np.asarray(b))
    return ((t > 0).sum(1) == 1).all() and ((t > 0).sum(0) == 1).all()


@pytest.mark.parametrize("backend", ["device", "sklearn"])
def test_kmeans_bic_recovers_clones(backend):
    mat, truth = _g1_matrix()
    cl = kmeans_cluster(mat, max_k=8, backend=backend, device="cpu")
    assert list(cl["cell_id"]) == list(mat.columns)
    assert cl["cluster_id"].nunique() == 3
    assert _same_partition(cl["cluster_id"], truth.loc[cl["cell_id"]].to_numpy())


def test_kmeans_fit_inertia_matches_sklearn():
    """Best-of-restarts inertia of the batched fit equals sklearn's on separable data."""
    import sklearn.cluster
    rng = np.random.default_rng(1)
    X = np.concatenate([rng.normal(m, 0.2, size=(50, 5)) for m in (0.0, 3.0, 6.0, 9.0)])
    _, _, inertia = kmeans_fit(X, 4, n_init=10, device="cpu")
    ref = sklearn.cluster.KMeans(n_clusters=4, init="k-means++", n_init=10, random_state=0).fit(X).inertia_
    assert np.isclose(inertia, ref, rtol=1e-9)


def test_clustered_labels_block_path_equals_general_path(monkeypatch):
    """scRT(clone_col=None): the G1/2 table's cluster_id column and the S cells' assigned
    clones from the per-cell-block fast paths equal the general paths' (label lookups per row,
    the reference's merge and per-cell assignment), dtypes included."""
    from scdna_replication_tools_amd import infer_scRT as isc
    from scdna_replication_tools_amd import prep
    from scdna_replication_tools_amd.simulator import simulate, to_long_form
    sim = simulate(n_s=24, n_g=45, n_bins=300, num_reads=300 * 183, seed=12, n_clones=3)
    s, g = to_long_form(sim, n_libs=1, copy_from="reads")
    s, g = s.drop(columns=["clone_id"]), g.drop(columns=["clone_id"])

    def run():
        sc = isc.scRT(s.copy(), g.copy(), clone_col=None, cn_prior_method="g1_clones", device="cpu")
        sc._pert_model()
        return sc
    fast = run()
    real = prep._block_layout
    monkeypatch.setattr(prep, "_block_layout", lambda *a, **k: None)
    slow = run()
    monkeypatch.setattr(prep, "_block_layout", real)
    pd.testing.assert_frame_equal(fast.cn_g1.reset_index(drop=True), slow.cn_g1.reset_index(drop=True))
    a = fast.cn_s.sort_values(["cell_id", "chr", "start"]).reset_index(drop=True)
    b = slow.cn_s.sort_values(["cell_id", "chr", "start"]).reset_index(drop=True)
    assert a["cluster_id"].dtype == b["cluster_id"].dtype
    np.testing.assert_array_equal(a["cluster_id"].to_numpy(), b["cluster_id"].to_numpy())
    assert a["chr"].map(type).eq(str).all() and b["chr"].map(type).eq(str).all()
