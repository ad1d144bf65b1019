"""Where finalize's time goes: on a bench-built shard after a few steps,
HIP events around repeated launches of pert_finalize, its shared half (bin sums, the pass's
ELBO / d/da partials, the priors' parameter terms, the global sums) and its per-cell half (the
cells' partial rows), each on the same state (read-only except for its own outputs).
    python tools/finalize_parts_probe.py [--cells 1250] [--reps 50]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cells", type=int, default=1250)
    ap.add_argument("--subdivide", type=int, default=1)
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    os.environ.setdefault("PERT_PLACEMENT", "0")
    from scdna_replication_tools_amd import _native as nat
    from scdna_replication_tools_amd.engine import EtaCodebook, PertShard
    from scdna_replication_tools_amd.init import init_params
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    data = bench.synth(a.cells, a.subdivide, seed=0, device=dev)
    reads = data["reads"].cpu().numpy()
    eta = EtaCodebook.from_states(data["cn"].cpu().numpy(), 1e6, bench.P)
    t_init = np.clip(data["tau"].cpu().numpy(), 0.05, 0.95)
    bm = np.zeros((1, bench.K + 1))
    bm[0, bench.K - 1] = 0.5
    libs = np.zeros(a.cells, int)
    init = init_params(2, reads, libs, 1, bench.P, bench.K, ploidy=eta.argmax_states().mean(0), t_init=t_init,
                       beta_means=bm, seed=0)
    sh = PertShard(2, reads, data["gc"], libs, 1, bench.P, bench.K, init, eta=eta, lamb=0.75, beta_means=bm,
                   device=dev)
    del data
    sh.run_svi(5, 10 ** 9, 0.0)
    s = torch.cuda.current_stream().cuda_stream
    lib = sh.lib
    calls = {"pert_finalize": lambda: lib.pert_finalize(ctypes.byref(sh._prob), ctypes.byref(sh._state), s),
             "pert_finalize_shared": lambda: lib.pert_finalize_shared(ctypes.byref(sh._prob),
                                                                      ctypes.byref(sh._state), s),
             "pert_finalize_cells": lambda: lib.pert_finalize_cells(ctypes.byref(sh._prob),
                                                                    ctypes.byref(sh._state), s)}
    out = {"cells": a.cells, "bins": sh.L, "bins_per_tile": sh.bins_per_tile}
    for rep in range(2):
        for name, fn in calls.items():
            nat.check(fn(), name)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                nat.check(fn(), name)
            e1.record()
            e1.synchronize()
            out.setdefault(name + "_us", []).append(round(1e3 * e0.elapsed_time(e1) / a.reps, 2))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
