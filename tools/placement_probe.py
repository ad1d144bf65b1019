"""Why some z / m / v placements stream fast: one process holds the C4
shard's pi state in N_SETS allocations, times the pass's own streams (pert_stream_ceiling) on
each, then runs REPS more ceiling launches per set in set order -- under rocprofv3 --pmc those
dispatches carry the counters, and tools/placement_pmc.py averages them over the fast and the
slow sets of the same process.  Prints one JSON line: per set its times (ms) and the set order
of the counter phase.
    python tools/placement_probe.py [--sets 12] [--reps 3] [--cells 10000]
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
    ap.add_argument("--sets", type=int, default=12)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--cells", type=int, default=10000)
    a = ap.parse_args()
    os.environ["PERT_PLACEMENT"] = "0"
    from scdna_replication_tools_amd import _native as nat
    from scdna_replication_tools_amd.engine import EtaCodebook, PertShard
    from scdna_replication_tools_amd.init import init_params
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    data = bench.synth(a.cells, 1, seed=0, device=dev)
    reads = data["reads"].cpu().numpy()
    eta = EtaCodebook.from_states(data["cn"].cpu().numpy(), 1e6, bench.P)
    t_init = np.clip(data["tau"].cpu().numpy(), 0.05, 0.95)
    bm = np.zeros((1, bench.K + 1))
    bm[0, bench.K - 1] = 0.5
    libs = np.zeros(a.cells, int)
    init = init_params(2, reads, libs, 1, bench.P, bench.K, ploidy=eta.argmax_states().mean(0), t_init=t_init,
                       beta_means=bm, seed=0)
    sh = PertShard(2, reads, data["gc"], libs, 1, bench.P, bench.K, init, eta=eta, lamb=0.75, beta_means=bm,
                   device=dev, placement=0)
    del data
    sets = [(sh.z_pi, sh.m_pi, sh.v_pi)]
    for _ in range(a.sets - 1):
        sets.append(tuple(torch.empty_like(sh.z_pi) for _ in range(3)))
    s = torch.cuda.current_stream().cuda_stream

    def launch():
        nat.check(sh.lib.pert_stream_ceiling(ctypes.byref(sh._prob), ctypes.byref(sh._state), s),
                  "pert_stream_ceiling")

    times = []
    for k, st in enumerate(sets):
        sh._set_pi_ptrs(*st)
        launch()
        ms = []
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            launch()
            e1.record()
            e1.synchronize()
            ms.append(e0.elapsed_time(e1))
        times.append(ms)
    # the counter phase: REPS launches per set, in set order
    for k, st in enumerate(sets):
        sh._set_pi_ptrs(*st)
        for _ in range(a.reps):
            launch()
    torch.cuda.synchronize()
    sh._set_pi_ptrs(*sets[0])
    cells = -(-a.cells // 64) * 64
    pattern_bytes = float(cells) * sh.L * (6.0 + 24.0 * sh.P)
    print(json.dumps({"sets": a.sets, "reps": a.reps, "times_ms": times,
                      "tbs": [round(pattern_bytes / (min(t) * 1e-3) / 1e12, 3) for t in times],
                      "timing_dispatches_per_set": 4,
                      "ptrs": [[int(t.data_ptr()) for t in st] for st in sets]}), flush=True)


if __name__ == "__main__":
    main()
