"""Host-side stage timings of the drop-in pipeline (no GPU needed): process_input_data,
consensus profiles, the eta builder, make_g1_g2_training_data and package_s_output at a
configuration's shape, on simulator long-form tables.

    python tools/host_prep_profile.py --cells 10000 [--prior g1_clones]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cells", type=int, default=2000)
    ap.add_argument("--prior", default="g1_clones")
    ap.add_argument("--subdivide", type=int, default=1)
    args = ap.parse_args()
    from scdna_replication_tools_amd import prep
    from scdna_replication_tools_amd.pert_model import MapTrace, pert_infer_scRT
    from scdna_replication_tools_amd.simulator import simulate, to_long_form
    t = {}
    tic = time.perf_counter()
    sim = simulate(n_s=args.cells, n_g=args.cells, subdivide=args.subdivide, num_reads=1e6, seed=0)
    df_s, df_g = to_long_form(sim, n_libs=1)
    t["simulate"] = time.perf_counter() - tic
    m = pert_infer_scRT(df_s, df_g, input_col='reads', clone_col='clone_id', cn_prior_method=args.prior,
                        device="cpu")
    tic = time.perf_counter()
    inp = m._prepare()
    t["process_input_data"] = time.perf_counter() - tic
    tic = time.perf_counter()
    profiles = prep.consensus_clone_profiles(m.cn_g1, m.cn_state_col, clone_col=m.clone_col, cell_col=m.cell_col,
                                             chr_col=m.chr_col, start_col=m.start_col,
                                             cn_state_col=m.cn_state_col, keys=inp.keys_g)
    t["consensus_profiles"] = time.perf_counter() - tic
    tic = time.perf_counter()
    etas = m._build_etas(inp, profiles)
    t["eta_builder"] = time.perf_counter() - tic
    tic = time.perf_counter()
    prep.make_g1_g2_training_data(inp.states_g, inp.reads_g, inp.libs_g)
    t["g1_g2_training_data"] = time.perf_counter() - tic
    tic = time.perf_counter()
    st = etas.argmax_states()
    t["argmax_states"] = time.perf_counter() - tic
    L, N = inp.reads_s.shape
    trace = MapTrace(cn=st.astype(np.int64), rep=np.zeros((L, N), np.float32), expose_u=np.ones(N, np.float32),
                     expose_rho=np.full(L, 0.5, np.float32), expose_a=np.array([10.0], np.float32),
                     expose_tau=np.full(N, 0.5, np.float32))
    tic = time.perf_counter()
    out, supp = m.package_s_output(m.cn_s, trace, m._axes(inp.cells_s, inp.keys_s), np.array([0.75], np.float32),
                                   [1.0] * 10, [2.0] * 10)
    t["package_s_output"] = time.perf_counter() - tic
    print(json.dumps({"cells": args.cells, "bins": L, "rows_s": len(df_s), "seconds": t}))


if __name__ == "__main__":
    main()
