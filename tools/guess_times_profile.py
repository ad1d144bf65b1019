"""Time the batched tau initialiser (tau_init.guess_times_batched, pert_model.py:426-457) on
the device for S-phase and G1/2 cells of a synthetic sample: the batched scan and the per-cell
sklearn path of the fragile cells separately.

    python tools/guess_times_profile.py [--cells 2000]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cells", type=int, default=2000)
    args = ap.parse_args()
    from scdna_replication_tools_amd import tau_init
    from scdna_replication_tools_amd.simulator import simulate
    sim = simulate(n_s=args.cells, n_g=args.cells, num_reads=1e6, seed=0)
    out = {}
    for name, reads, cn in (("S", sim.reads_s, sim.cn_s), ("G", sim.reads_g, sim.cn_g)):
        for rep in range(2):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            tau_init.guess_times_batched(reads, cn, 6, device="cuda")
            torch.cuda.synchronize()
            out["{}_{}".format(name, rep)] = {"seconds": time.perf_counter() - t0,
                                              "fragile": int(len(tau_init.guess_times_batched.last_fragile))}
        x = torch.as_tensor(np.asarray(reads, np.float32), device="cuda")
        st = torch.as_tensor(np.asarray(cn, np.float32), device="cuda")
        norm = x / torch.where(st > 0.0, st, torch.full_like(st, 0.5))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        tau_init.binarization_fraction(norm, return_fragile=True, return_minor=True)
        torch.cuda.synchronize()
        out[name + "_scan_only"] = time.perf_counter() - t0
    print(json.dumps(out))


if __name__ == "__main__":
    main()
