"""Time the tau initialiser's exact host path (tau_init.exact_fractions, called by
guess_times_batched for the flagged cells) with 1..16 threads at a config's size, and check
that every thread count gives the same t_init.
usage: python tools/exact_threads_probe.py [--cells 10000] [--bins 5451]"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scdna_replication_tools_amd import tau_init  # noqa: E402
from scdna_replication_tools_amd.simulator import simulate  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cells", type=int, default=10000)
    ap.add_argument("--bins", type=int, default=5451)
    ap.add_argument("--threads", default="1,2,4,8,16")
    a = ap.parse_args()
    sim = simulate(n_s=a.cells, n_g=1, n_bins=a.bins, num_reads=1e6, seed=0)
    reads, states = sim.reads_s.astype(np.float32), sim.cn_s
    print("simulated", reads.shape, "affinity cores", len(os.sched_getaffinity(0)), flush=True)
    tau_init.guess_times_batched(reads, states, 6, device="cuda")          # warm-up (kernel load)
    ref = None
    for nt in [int(x) for x in a.threads.split(",")]:
        t0 = time.perf_counter()
        t = tau_init.guess_times_batched(reads, states, 6, device="cuda", n_threads=nt)[0]
        dt = time.perf_counter() - t0
        same = ref is None or np.array_equal(t, ref)
        ref = t if ref is None else ref
        print(nt, "threads: total {:.3f} s".format(dt), dict(tau_init.guess_times_batched.last_timings),
              "same t_init:", same, flush=True)


if __name__ == "__main__":
    main()
