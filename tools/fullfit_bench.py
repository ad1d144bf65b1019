"""Full-fit wall clock of the drop-in pipeline ("full two-step fit
wall-clock (steps 1+2; step 3 reported separately)") on simulator data.

    python tools/fullfit_bench.py --config c3 [--max-iter 2000] [--n-jobs 16]

Prints one JSON line with per-phase seconds (pert_infer_scRT.timings), iteration
counts, per-step milliseconds and decode accuracy against the simulator's truth.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import pandas as pd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CONFIGS = {"c1": (400, 271, 1), "c2": (2000, None, 1), "c3": (2000, None, 1), "c4": (10000, None, 1),
           "c5": (2000, None, 25)}
# c2: BASELINE configs[1] stand-in (polyclonal sample, clones unknown): C3-sized synthetic data
# through scRT(clone_col=None).infer('pert') -- KMeans + BIC clustering of the G1/2 cells first.


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--max-iter", type=int, default=2000)
    ap.add_argument("--min-iter", type=int, default=100)
    ap.add_argument("--n-jobs", type=int, default=16)
    ap.add_argument("--prior", default="g1_clones")
    ap.add_argument("--no-step3", action="store_true")
    ap.add_argument("--cpu-sample-cells", type=int, default=64,
                    help="oracle per-step timing sample (0: skip the CPU extrapolation)")
    args = ap.parse_args()
    import torch
    # under torch.distributed.run (WORLD_SIZE > 1): the fit cell-sharded over the ranks
    # (pert_model._Dist); PERT_DIST_BACKEND=gloo with PERT_NATIVE_COMM=host rehearses an
    # N-GPU node's C loop with the ranks sharing GPU 0.  Rank 0 prints the record.
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    fit_kw = {}
    if world > 1:
        import torch.distributed as dist
        backend = os.environ.get("PERT_DIST_BACKEND", "nccl")
        dev = 0 if backend == "gloo" else int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(dev)
        dist.init_process_group(backend)
        fit_kw["device"] = "cuda:{}".format(dev)
    from scdna_replication_tools_amd.pert_model import pert_infer_scRT
    from scdna_replication_tools_amd.simulator import simulate, to_long_form
    n, nb, sub = CONFIGS[args.config]
    t0 = time.perf_counter()
    sim = simulate(n_s=n, n_g=n, n_bins=nb, subdivide=sub, num_reads=1e6, seed=0)
    df_s, df_g = to_long_form(sim, n_libs=1, copy_from="reads" if args.config == "c2" else "state")
    t_sim = time.perf_counter() - t0
    print("simulated {} + {} cells x {} bins in {:.1f} s".format(n, n, sim.n_bins, t_sim), file=sys.stderr, flush=True)
    torch.zeros(1, device="cuda")
    # a heartbeat on stderr while the fit runs (a GPU command silent for minutes is taken as hung)
    import threading
    t_fit = time.perf_counter()
    beat = threading.Event()

    def heartbeat():
        while not beat.wait(20.0):
            print("... fit running {:.0f} s".format(time.perf_counter() - t_fit), file=sys.stderr, flush=True)
    threading.Thread(target=heartbeat, daemon=True).start()
    import contextlib
    fit_stdout = contextlib.redirect_stdout(sys.stderr)          # the fit's own prints (convergence lines)
    fit_stdout.__enter__()
    if args.config == "c2":
        from scdna_replication_tools_amd.infer_scRT import scRT
        t0 = time.perf_counter()
        sc = scRT(df_s.drop(columns=["clone_id"]), df_g.drop(columns=["clone_id"]), clone_col=None,
                  cn_prior_method=args.prior, max_iter=args.max_iter, min_iter=args.min_iter,
                  run_step3=not args.no_step3, n_jobs=args.n_jobs)
        cn_s_out, supp_s, cn_g1_out, supp_g1 = sc.infer(level='pert')
        m = sc.model
        m.timings["cluster_assign"] = time.perf_counter() - t0 - m.timings["total"]
        truth = df_g.drop_duplicates("cell_id").set_index("cell_id")["clone_id"]
        cl = sc.clusters.set_index("cell_id")["cluster_id"]
        ct = pd.crosstab(cl.to_numpy(), truth.loc[cl.index].to_numpy())
        clusters_ok = bool(((ct > 0).sum(1) == 1).all() and ((ct > 0).sum(0) == 1).all())
    else:
        m = pert_infer_scRT(df_s, df_g, input_col='reads', clone_col='clone_id', cn_prior_method=args.prior,
                            max_iter=args.max_iter, min_iter=args.min_iter, run_step3=not args.no_step3,
                            n_jobs=args.n_jobs, **fit_kw)
        cn_s_out, supp_s, cn_g1_out, supp_g1 = m.run_pert_model()
        clusters_ok = None
    beat.set()
    print("fit done: {}".format(m.timings), file=sys.stderr, flush=True)
    fit_stdout.__exit__(None, None, None)
    acc_cn = float((cn_s_out["model_cn_state"] == cn_s_out["true_somatic_cn"]).mean())
    acc_rep = float((cn_s_out["model_rep_state"] == cn_s_out["true_rep"]).mean())
    tm = m.timings
    rec = {"config": args.config, "cells_s": n, "cells_g": n, "bins": sim.n_bins, "prior": args.prior,
           "simulate_s": t_sim, "timings_s": tm, "iters": m.iters,
           "ms_per_step": {k: 1e3 * tm[k] / max(1, m.iters[k]) for k in m.iters},
           "fit_steps12_s": tm["total"] - sum(tm.get(k, 0.0) for k in ("prep_step3", "step3", "decode_package_g")),
           "acc_cn": acc_cn, "acc_rep": acc_rep}
    if clusters_ok is not None:
        rec["clusters_match_truth"] = clusters_ok
        rec["n_clusters"] = int(sc.clusters["cluster_id"].nunique())
    if world > 1:
        rec["ranks"] = {"world": world, "backend": os.environ.get("PERT_DIST_BACKEND", "nccl"),
                        "native_comm": os.environ.get("PERT_NATIVE_COMM", "1"), "launched": m.launched}
        import torch.distributed as dist
        dist.destroy_process_group()
        if rank != 0:
            return
    if args.cpu_sample_cells > 0:
        print("timing the CPU oracle on {} cells".format(args.cpu_sample_cells), file=sys.stderr, flush=True)
        from bench import cpu_extrapolation           # bench.py's cpu_baseline leg (the oracle)
        rec["cpu_extrapolated"] = cpu_extrapolation(sim, m.iters, args.cpu_sample_cells)
        fit12 = rec["cpu_extrapolated"]["step1_s"] + rec["cpu_extrapolated"]["step2_s"]
        rec["speedup_fit_steps12_vs_cpu"] = fit12 / rec["fit_steps12_s"]
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
