"""Where the batched tau initialiser's time goes at C4 (10 k cells x 5,451 bins) on one MI355X:
the host normalisation (cn_normalise), the copy to the device, the tau_binarize_kernel launch
(synchronised) and the copies back -- each timed alone after a warm-up.

    python tools/tau_parts_probe.py [--cells 10000]
Prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cells", type=int, default=10000)
    a = ap.parse_args()
    import numpy as np
    import torch
    from scdna_replication_tools_amd import tau_init
    from scdna_replication_tools_amd.simulator import simulate
    sim = simulate(n_s=a.cells, n_g=16, num_reads=1e6, seed=0)
    reads = np.ascontiguousarray(sim.reads_s, dtype=np.float32)
    states = np.ascontiguousarray(sim.cn_s)
    dev = torch.device("cuda", 0)
    out = {"cells": a.cells}

    def timed(name, f, reps=3):
        f()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            r = f()
            torch.cuda.synchronize()
        out[name] = round((time.perf_counter() - t0) / reps, 4)
        return r

    norm = timed("cn_normalise", lambda: torch.from_numpy(tau_init.cn_normalise(reads, states)))
    nd = timed("to_device", lambda: norm.to(dev))
    res = timed("binarization_fraction", lambda: tau_init.binarization_fraction(nd, return_fragile=True,
                                                                                return_minor=True))
    timed("results_to_host", lambda: [x.cpu() for x in res])
    timed("guess_times_batched", lambda: tau_init.guess_times_batched(reads, states, device=dev), reps=1)
    out["last_timings"] = tau_init.guess_times_batched.last_timings
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
