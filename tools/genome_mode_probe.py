"""Is a G1 cell's step-3 mode (tau ~ 0 vs tau ~ 1: a G1 profile fits as unreplicated, or as fully
replicated with u about halved) decided by rounding?  Runs the genome-length fixture's fit
(tests/_configs.py genome_tables, the reference's defaults) with three summation orders of the
same arithmetic -- the default pass, another tile length (other per-cell partial sums) and the
variant-0 enumerated pass -- and prints, per run, the G1 cells fitted at tau > 0.5 and the
agreement with the committed fp32 oracle chain (tests/golden/genome_chain_oracle.npz).
usage: python tools/genome_mode_probe.py"""
import functools
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from scdna_replication_tools_amd import engine  # noqa: E402
from tests._chain import product_arrays  # noqa: E402
from tests._configs import genome_scrt, genome_tables  # noqa: E402


def run(label, **shard_kw):
    orig = engine.PertShard.__init__
    if shard_kw:
        engine.PertShard.__init__ = functools.partialmethod(orig, **shard_kw)
    try:
        s, g, _ = genome_tables()
        sc = genome_scrt(s, g)
        out = sc.infer(level='pyro')
        prod = product_arrays(sc.model, *out)
    finally:
        engine.PertShard.__init__ = orig
    fx = dict(np.load(os.path.join(ROOT, "tests", "golden", "genome_chain_oracle.npz")))
    hi = [int(i) for i in np.flatnonzero(prod["tau_g"] > 0.5)]
    rec = {"run": label, "iters": [len(prod["losses_g"]), len(prod["losses_s"]), len(prod["losses_s2"])],
           "g1_cells_tau_gt_half": hi, "oracle_g1_cells_tau_gt_half": [int(i) for i in np.flatnonzero(fx["tau_g"] > 0.5)],
           "cn_g_agree": float(((prod["cn_g"] == fx["cn_g"]) & (prod["rep_g"] == fx["rep_g"])).mean()),
           "cn_s_agree": float(((prod["cn_s"] == fx["cn_s"]) & (prod["rep_s"] == fx["rep_s"])).mean())}
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    run("default")
    run("bins_per_tile=24", bins_per_tile=24)
    run("variant 0", variant=0)
