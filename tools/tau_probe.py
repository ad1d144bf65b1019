"""Time the tau initialiser (tau_init.guess_times_batched) on the GPU at a config's size:
the HIP k-means / EM launch, the levels / scan stage and the exact host path, separately.
usage: python tools/tau_probe.py [--cells 10000] [--bins 5451]"""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scdna_replication_tools_amd import tau_init  # noqa: E402
from scdna_replication_tools_amd.simulator import simulate  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cells", type=int, default=10000)
    ap.add_argument("--bins", type=int, default=5451)
    a = ap.parse_args()
    sim = simulate(n_s=a.cells, n_g=1, n_bins=a.bins, num_reads=1e6, seed=0)
    reads, states = sim.reads_s.astype(np.float32), sim.cn_s.astype(np.float32)
    print("simulated", reads.shape, flush=True)
    x, st = torch.as_tensor(reads), torch.as_tensor(states)
    norm = (x / torch.where(st > 0.0, st, (torch.ones(x.shape) * 0.5).type(torch.float32))).cuda()
    torch.cuda.synchronize()
    for rep in range(2):
        t0 = time.perf_counter()
        res = tau_init.binarize_native(norm)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        flags = [(int(r["fragile"].sum()), int(r["pp"].sum()), int(r["scan"].sum())) for r in res]
        print("one-launch pass {:.4f} s, (fragile, kmeans++, scan) per run {}".format(t1 - t0, flags), flush=True)
    t0 = time.perf_counter()
    frac, lab_unsure, near, lab = tau_init.binarization_fraction(norm, return_fragile=True, return_minor=True)
    torch.cuda.synchronize()
    redo = np.flatnonzero((lab_unsure | near).cpu().numpy())
    print("batched pass {:.3f} s: k-means unsure {}, scan near {}, to the exact path {}".format(
        time.perf_counter() - t0, int(lab_unsure.sum()), int(near.sum()), redo.size), flush=True)
    sub = redo[:64]
    labels = lab[:, torch.as_tensor(sub, device=lab.device)].T.to(torch.int8).cpu().numpy()
    labels[lab_unsure[torch.as_tensor(sub, device=lab.device)].cpu().numpy()] = -1
    t0 = time.perf_counter()
    tau_init.exact_fractions(norm[:, torch.as_tensor(sub, device=norm.device)].cpu().numpy(), labels,
                             n_threads=tau_init.default_threads())
    dt = time.perf_counter() - t0
    print("exact path: {} cells in {:.3f} s ({} k-means on the host) -> {:.1f} s for all {}".format(
        sub.size, dt, int((labels[:, 0] < 0).sum()), dt * redo.size / max(sub.size, 1), redo.size), flush=True)
    if redo.size > 2000:
        return
    t0 = time.perf_counter()
    tau_init.guess_times_batched(reads, states, 6, device="cuda")
    print("guess_times_batched {:.3f} s {}".format(time.perf_counter() - t0, tau_init.guess_times_batched.last_timings),
          flush=True)


if __name__ == "__main__":
    main()
