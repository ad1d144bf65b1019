"""Per-rank host work of a sharded fit at a genome-length size.

The public entry point ``pert_infer_scRT(...).run_pert_model()`` on configs[2]-shaped synthetic
tables (``--cells`` S + G1/2 cells x 5,451 bins, 3 clones) once on one rank and once on two
gloo ranks sharing the GPU, with a warm-up fit first in every process (first-use costs
excluded).  Prints each run's tau-initialiser cell counts and the helper's durations
(``timings["helper_guess_times_s"]`` / ``["helper_guess_times_g"]``): a sharded rank makes the
CN prior, runs guess_times and draws the initial values for its own cells only.

    python tools/api_ranks_timing.py [--cells 2000] [--max-iter 200]
"""
import argparse
import json
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

KEYS = ("helper_guess_times_s", "helper_guess_times_g", "helper_priors", "prep", "total")


def _tables(cells):
    from scdna_replication_tools_amd.simulator import simulate, to_long_form
    sim = simulate(n_s=cells, n_g=cells, n_clones=3, num_reads=1e6, seed=3)
    return to_long_form(sim, n_libs=1)


def _fit(s, g, max_iter, device):
    from scdna_replication_tools_amd.pert_model import pert_infer_scRT
    m = pert_infer_scRT(s.copy(), g.copy(), input_col='reads', clone_col='clone_id', cn_prior_method='g1_clones',
                        max_iter=max_iter, min_iter=max_iter, device=device, log_steps=False)
    m.run_pert_model()
    t = {k: m.timings.get(k) for k in KEYS}
    t["tau_cells_s"] = m.timings.get("tau_init_s", {}).get("cells")
    t["tau_exact_cells_s"] = m.timings.get("tau_init_s", {}).get("exact_cells")
    t["tau_cells_g"] = m.timings.get("tau_init_g", {}).get("cells")
    t["tau_exact_cells_g"] = m.timings.get("tau_init_g", {}).get("exact_cells")
    return t


def _worker(rank, world, port, cells, max_iter, out):
    import torch
    import torch.distributed as dist
    import contextlib
    import io
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:{}".format(port), rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        s, g = _tables(cells)
        with contextlib.redirect_stdout(io.StringIO()):
            _fit(s, g, 20, "cuda:0")                                 # warm-up (first-use costs)
            t = _fit(s, g, max_iter, "cuda:0")
        with open(out.format(rank), "w") as fh:
            json.dump(t, fh)
    finally:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cells", type=int, default=2000)
    ap.add_argument("--max-iter", type=int, default=200)
    a = ap.parse_args()
    import contextlib
    import io
    import torch
    import torch.multiprocessing as mp
    out = os.path.join(ROOT, "gpurun_out", "api_ranks_timing_rank{}.json")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    t0 = time.time()
    ctx = mp.spawn(_worker, args=(2, port, a.cells, a.max_iter, out), nprocs=2, join=False)
    while not ctx.join(timeout=10):
        print("... two ranks running {:.0f} s".format(time.time() - t0), flush=True)
        if time.time() - t0 > 400:
            for p in ctx.processes:
                if p.is_alive():
                    p.kill()
            raise SystemExit("two-rank fit did not finish")
    ranks = [json.load(open(out.format(r))) for r in range(2)]
    s, g = _tables(a.cells)
    with contextlib.redirect_stdout(io.StringIO()):
        _fit(s, g, 20, "cuda:0")
        one = _fit(s, g, a.max_iter, "cuda:0")
    print(json.dumps({"cells": a.cells, "bins": 5451, "max_iter": a.max_iter, "one_rank": one,
                      "rank0": ranks[0], "rank1": ranks[1]}), flush=True)


if __name__ == "__main__":
    main()
