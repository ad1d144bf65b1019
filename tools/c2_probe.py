"""Where the configs[1] stand-in (polyclonal, clone_col=None) spends the time before the fit:
the G1/2 pivot, KMeans + BIC for k = 2..20 (per k), the consensus profiles and the S-cell
assignment (infer_scRT.py:127-148), timed on the GPU box.
usage: python tools/c2_probe.py"""
import os
import sys
import time

import numpy as np
import pandas as pd
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from scdna_replication_tools_amd import cncluster, prep
    from scdna_replication_tools_amd.infer_scRT import assign_s_to_clones
    from scdna_replication_tools_amd.simulator import simulate, to_long_form
    sim = simulate(n_s=2000, n_g=2000, n_bins=5451, num_reads=1e6, seed=0)
    df_s, df_g = to_long_form(sim, n_libs=1, copy_from="reads")
    df_s, df_g = df_s.drop(columns=["clone_id"]), df_g.drop(columns=["clone_id"])
    torch.zeros(1, device="cuda")
    t0 = time.perf_counter()
    piv = prep.pivot_cells_by_loci(df_g, "copy", "cell_id", "chr", "start")
    g1_mat = pd.DataFrame(piv.values, columns=pd.Index(piv.cells, name="cell_id"),
                          index=pd.MultiIndex.from_arrays([piv.loci_chr, piv.loci_start], names=["chr", "start"]))
    t1 = time.perf_counter()
    print("pivot {:.3f} s".format(t1 - t0), flush=True)
    X = np.asarray(g1_mat.T.values, dtype=np.float64)
    for k in (2, 3, 5, 10, 20):
        t = time.perf_counter()
        C, lab, _ = cncluster.kmeans_fit(X, k, n_init=10, device="cuda")
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        cncluster.compute_bic(C, lab, X)
        print("k={:2d}: kmeans_fit {:.3f} s, compute_bic {:.3f} s".format(k, t2 - t, time.perf_counter() - t2), flush=True)
    t = time.perf_counter()
    cl = cncluster.kmeans_cluster(g1_mat, max_k=20, device="cuda")
    t2 = time.perf_counter()
    print("kmeans_cluster k=2..20 {:.3f} s -> {} clusters".format(t2 - t, cl.cluster_id.nunique()), flush=True)
    lut = pd.Series(cl["cluster_id"].to_numpy(), index=cl["cell_id"].to_numpy())
    df_g = df_g.assign(cluster_id=df_g["cell_id"].map(lut).astype(np.int64))
    t = time.perf_counter()
    prof = prep.consensus_clone_profiles(df_g, "copy", clone_col="cluster_id", cell_col="cell_id", chr_col="chr",
                                         start_col="start", cn_state_col="state")
    t2 = time.perf_counter()
    assign_s_to_clones(df_s, prof, col_name="copy", clone_col="cluster_id", cell_col="cell_id", chr_col="chr",
                       start_col="start")
    print("consensus {:.3f} s, assign_s_to_clones {:.3f} s".format(t2 - t, time.perf_counter() - t2), flush=True)


if __name__ == "__main__":
    main()
