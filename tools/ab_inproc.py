"""In-process A/B of two builds of libpert_hip.so on the same shard: both builds' shards live
in one process and alternate in short blocks of SVI steps, so clock / thermal drift of the box
(which moves separate bench runs by 5-10 %) hits both arms alike.

    python tools/ab_inproc.py --lib-b path/to/other.so [--lib-a default.so] [--cells 10000]
Prints the median enumerated-pass time of each arm and B/A.  The arms' buffers sit at different
addresses, which on some boxes alone moves one arm by up to ~10 % (same build in both arms:
B/A 0.89 on one box, 1.002 on another), so a result is only read with the arms also swapped.
"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib-a", default=os.path.join(ROOT, "scdna_replication_tools_amd", "libpert_hip.so"))
    ap.add_argument("--lib-b", required=True)
    ap.add_argument("--cells", type=int, default=10000)
    ap.add_argument("--rounds", type=int, default=12)
    ap.add_argument("--steps", type=int, default=4, help="SVI steps per block")
    ap.add_argument("--variant-b", type=int, default=0)

    args = ap.parse_args()
    import bench
    from scdna_replication_tools_amd import _native as nat
    from scdna_replication_tools_amd.engine import EtaCodebook, PertShard
    from scdna_replication_tools_amd.init import init_params
    dev = torch.device("cuda", 0)
    data = bench.synth(args.cells, 1, 0, dev)
    reads = data["reads"].cpu().numpy()
    gc = data["gc"]
    eta = EtaCodebook.from_states(data["cn"].cpu().numpy(), 1e6, 13)
    bm = np.zeros((1, 5))
    bm[0, 3] = 0.5
    init = init_params(2, reads, np.zeros(args.cells, int), 1, 13, 4, ploidy=eta.argmax_states().mean(0),
                       t_init=np.clip(data["tau"].cpu().numpy(), 0.05, 0.95), beta_means=bm, seed=0)
    del data
    arms = {}
    for name, path, var in (("A", args.lib_a, 0), ("B", args.lib_b, args.variant_b)):
        sh = PertShard(2, reads, gc, np.zeros(args.cells, int), 1, 13, 4, init,
                       eta=eta, lamb=0.75, beta_means=bm, device=dev, lib=nat.load(path), variant=var)
        sh.run_svi(2, 10 ** 9, 0.0)                                  # warm-up
        arms[name] = (sh, [])
    for _ in range(args.rounds):
        for name in ("A", "B"):
            sh, times = arms[name]
            sh.pass_events = []
            sh.run_svi(args.steps, 10 ** 9, 0.0)
            times.extend(a.elapsed_time(b) for a, b in sh.pass_events)
            sh.pass_events = None
    ma = float(np.median(arms["A"][1]))
    mb = float(np.median(arms["B"][1]))
    print("A {:.4f} ms  B {:.4f} ms  B/A {:.4f}  (median of {} passes each, LT {} / {})".format(
        ma, mb, mb / ma, len(arms["A"][1]), arms["A"][0].bins_per_tile, arms["B"][0].bins_per_tile), flush=True)


if __name__ == "__main__":
    main()
