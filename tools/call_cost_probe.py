"""Fixed cost of one PertShard.run_svi call: the 1,250-cell shard (C4's
per-rank work at N = 8) with the library's one-rank RCCL communicator, as bench.py builds it;
run_svi(K) for K = 8 / 20 / 200 repeatedly, the wall time split into the C call
(pert_svi_run_sharded) and the Python around it, against K x the per-step time of a long call.
    python tools/call_cost_probe.py [--cells 1250] [--reps 5]
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cells", type=int, default=1250)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--comm", default="rccl", choices=["rccl", "none"])
    a = ap.parse_args()
    from scdna_replication_tools_amd.engine import EtaCodebook, PertShard, RcclComm
    from scdna_replication_tools_amd.init import init_params
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    data = bench.synth(a.cells, 1, seed=0, device=dev)
    reads = data["reads"].cpu().numpy()
    states = data["cn"].cpu().numpy()
    eta = EtaCodebook.from_states(states, 1e6, bench.P)
    t_init = np.clip(data["tau"].cpu().numpy(), 0.05, 0.95)
    bm = np.zeros((1, bench.K + 1))
    bm[0, bench.K - 1] = 0.5
    libs = np.zeros(a.cells, int)
    init = init_params(2, reads, libs, 1, bench.P, bench.K, ploidy=eta.argmax_states().mean(0), t_init=t_init,
                       beta_means=bm, seed=0)
    comm = RcclComm.world1() if a.comm == "rccl" else None
    sh = PertShard(2, reads, data["gc"], libs, 1, bench.P, bench.K, init, eta=eta, lamb=0.75, beta_means=bm,
                   device=dev, comm=comm)
    # the C call's own duration: wrap the bound function
    fn_name = "pert_svi_run_sharded" if comm is not None else "pert_svi_run"
    lib = sh._lib_chunk
    orig = getattr(lib, fn_name)
    c_times = []

    class Timed:
        def __call__(self, *args):
            t0 = time.perf_counter()
            rc = orig(*args)
            c_times.append(time.perf_counter() - t0)
            return rc
    setattr(lib, fn_name, Timed())
    sh.reserve_svi(4096)
    sh.run_svi(200, 10 ** 9, 0.0)
    out = {}
    for K in (8, 20, 200, 20, 8):
        walls, cs = [], []
        for _ in range(a.reps):
            torch.cuda.synchronize()
            c_times.clear()
            t0 = time.perf_counter()
            sh.run_svi(K, 10 ** 9, 0.0)
            torch.cuda.synchronize()
            walls.append(time.perf_counter() - t0)
            cs.append(c_times[0])
        out.setdefault(K, []).append({"wall_ms": 1e3 * float(np.median(walls)), "c_call_ms": 1e3 * float(np.median(cs))})
        print("K={:4d}: wall {:.3f} ms ({:.4f} ms/step), C call {:.3f} ms, Python around it {:.3f} ms".format(
            K, 1e3 * np.median(walls), 1e3 * np.median(walls) / K, 1e3 * np.median(cs),
            1e3 * (np.median(walls) - np.median(cs))), flush=True)
    per_step = out[200][0]["wall_ms"] / 200
    for K in (8, 20):
        w = np.mean([r["wall_ms"] for r in out[K]])
        print("K={}: fixed cost per call {:.3f} ms (wall - K x {:.4f} ms/step of the K = 200 call)".format(
            K, w - K * per_step, per_step))
    print(json.dumps({str(k): v for k, v in out.items()}))
    setattr(lib, fn_name, orig)
    if comm is not None:
        comm.close()


if __name__ == "__main__":
    main()
