"""The step-2 pass on the product fit's own C4 inputs (numpy simulator -> pert_infer_scRT prep ->
g1_clones eta -> tau initialiser -> PertShard), timed like bench.py times its synthetic shard:
mean pass time by HIP events over K steps and the pass's pattern ceiling on the same shard.
usage: python tools/fit_pass_probe.py [--steps 30]"""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from scdna_replication_tools_amd import prep
    from scdna_replication_tools_amd._native import KIND_STEP2
    from scdna_replication_tools_amd.engine import PertShard
    from scdna_replication_tools_amd.init import init_params
    from scdna_replication_tools_amd.pert_model import pert_infer_scRT
    from scdna_replication_tools_amd.simulator import simulate, to_long_form
    from scdna_replication_tools_amd.tau_init import guess_times_batched
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=30)
    a = ap.parse_args()
    sim = simulate(n_s=10000, n_g=10000, n_bins=5451, num_reads=1e6, seed=0)
    df_s, df_g = to_long_form(sim, n_libs=1, copy_from="state")
    m = pert_infer_scRT(df_s, df_g, input_col='reads', clone_col='clone_id', cn_prior_method='g1_clones',
                        log_steps=False)
    inp = m._prepare()
    prof = prep.consensus_clone_profiles(m.cn_g1, m.cn_state_col, keys=inp.keys_g)
    eta = m._build_etas(inp, prof)
    t_init = guess_times_batched(inp.reads_s, eta.argmax_states(), 6, device="cuda")[0]
    bm = np.zeros((1, m.K + 1), np.float32)
    init = init_params(KIND_STEP2, inp.reads_s, inp.libs_s, 1, m.P, m.K, ploidy=eta.ploidy(), t_init=t_init,
                       beta_means=bm)
    sh = PertShard(KIND_STEP2, inp.reads_s, inp.gc, inp.libs_s, 1, m.P, m.K, init, eta=eta, lamb=0.7,
                   beta_means=bm, device="cuda")
    print("shard: {} cells x {} bins, LT {}, eta rows {}".format(sh.N, sh.L, sh.bins_per_tile, eta.table.shape[0]),
          flush=True)
    sh.run_svi(5, 10 ** 9, 0.0)
    sh.pass_events = []
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    sh.run_svi(a.steps, 10 ** 9, 0.0)
    torch.cuda.synchronize()
    step_ms = (time.perf_counter() - t0) / a.steps * 1e3
    kern = float(np.mean([x.elapsed_time(y) for x, y in sh.pass_events]))
    sh.pass_events = None
    ceil = sh.stream_ceiling_ms()
    print("fit inputs: step {:.4f} ms, pass {:.4f} ms, pattern ceiling {:.4f} ms ({:.3f})".format(
        step_ms, kern, ceil, ceil / kern), flush=True)


if __name__ == "__main__":
    main()
