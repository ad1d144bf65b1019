"""Golden vectors from the REFERENCE's own host functions, run in the build container only
(the reference does not travel to the GPU box; the committed .npz is data).

Importable here without the missing third-party packages:
``compute_consensus_clone_profiles`` (compute_consensus_clone_profiles.py:42-88).  Its
ploidy filter (``add_cell_ploidies``, :30-39) raises on this stack (scipy >= 1.11 returns a
scalar from ``stats.mode``: ``mode(...)[0][0]`` -> IndexError) and ``assign_s_to_clones``
uses ``DataFrame.iteritems`` (removed in pandas 2), so only the ``cn_state_col=None`` path
-- the per-(locus, clone) median pivot -- is pinned here.

    python tests/golden/make_reference_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
REF = "/root/reference/scdna_replication_tools"


def main():
    from scdna_replication_tools_amd.simulator import simulate, to_long_form
    sys.path.insert(0, REF)
    import compute_consensus_clone_profiles as ccp                     # the reference module
    sim = simulate(n_s=6, n_g=21, n_bins=180, num_reads=400 * 180, seed=11)
    _, df_g = to_long_form(sim, copy_from="reads")
    rng = np.random.default_rng(2)
    df_g = df_g.sample(frac=1.0, random_state=4).reset_index(drop=True)   # unsorted input rows
    drop = rng.uniform(size=len(df_g)) < 0.03                            # a few missing (cell, locus) rows
    df_g = df_g[~drop].reset_index(drop=True)
    df_g.loc[df_g.index[:5], "clone_id"] = "None"                        # rows of the removed 'None' clone
    prof = ccp.compute_consensus_clone_profiles(df_g.copy(), "copy", clone_col="clone_id", cell_col="cell_id",
                                                chr_col="chr", start_col="start", cn_state_col=None)
    out = dict(cell_id=df_g["cell_id"].to_numpy().astype("U"), chr=df_g["chr"].to_numpy().astype("U"),
               start=df_g["start"].to_numpy(np.int64), clone_id=df_g["clone_id"].to_numpy().astype("U"),
               copy=df_g["copy"].to_numpy(np.float64),
               prof_values=prof.to_numpy(np.float64),
               prof_chr=np.asarray(prof.index.get_level_values(0)).astype("U"),
               prof_start=np.asarray(prof.index.get_level_values(1), dtype=np.int64),
               prof_clones=np.asarray(prof.columns).astype("U"))
    path = os.path.join(HERE, "consensus_reference.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, prof.shape)


if __name__ == "__main__":
    main()
