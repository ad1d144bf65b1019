"""Step 2 of the genome-length chain ALONE on the GPU, from the fixture's step-1 sites (lambda,
beta_means) and t_init -- the GPU counterpart of tools/stop_probe.py (which runs the same
step on the CPU oracle).  Separates the two sources of a stopping-iteration difference in
tests/test_gpu_chain.py's genome test: step 1's outputs (which step 2 starts from) and step 2's
own arithmetic.  Test infrastructure: reads the committed fixture only.

    python tools/gpu_step2_probe.py [--out gpurun_out/step2_probe.npz] [--step1-from file.npz]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from tests._configs import genome_scrt, genome_tables  # noqa: E402

FIXTURE = os.path.join(ROOT, "tests", "golden", "genome_chain_oracle.npz")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--step1-from", default=None, help="an .npz with lam (and beta_means) to start from")
    a = ap.parse_args()
    from scdna_replication_tools_amd import prep
    from scdna_replication_tools_amd.init import init_params
    from scdna_replication_tools_amd.pert_model import KIND_STEP2, _Dist
    fx = dict(np.load(FIXTURE))
    s, g, _ = genome_tables()
    m = genome_scrt(s, g)._pert_model()
    inp = m._prepare()
    profiles = prep.consensus_clone_profiles(m.cn_g1, m.cn_state_col, clone_col=m.clone_col, cell_col=m.cell_col,
                                             chr_col=m.chr_col, start_col=m.start_col, cn_state_col=m.cn_state_col,
                                             keys=inp.keys_g)
    etas = m._build_etas(inp, profiles)
    lam = np.asarray(fx["lam"], np.float32).reshape(-1)
    bm = np.asarray(fx["beta_means"], np.float32)
    if a.step1_from:
        alt = dict(np.load(a.step1_from))
        lam = np.asarray(alt["lam"], np.float32).reshape(-1)
        if "beta_means" in alt:
            bm = np.asarray(alt["beta_means"], np.float32).reshape(bm.shape)
    t_init = np.asarray(fx["t_init_s"], np.float32)
    init2 = init_params(KIND_STEP2, inp.reads_s, inp.libs_s, m.L, m.P, m.K, ploidy=etas.ploidy(), t_init=t_init,
                        beta_means=bm, seed=m.seed, method=m.init_method)
    s2 = m._shard(KIND_STEP2, _Dist(None), inp.reads_s, inp.libs_s, init2, eta=etas, lamb=float(lam[0]), beta_means=bm)
    losses = np.asarray(m._svi(s2, m.max_iter, m.min_iter, "step2"), np.float64)
    ref = np.asarray(fx["losses_s"], np.float64)
    n = min(len(losses), len(ref))
    dev = np.abs(losses[:n] - ref[:n])
    out = {"stop": int(len(losses)), "fixture_stop": int(len(ref)), "dev_first": float(dev[0]),
           "dev_max": float(dev.max()), "dev_argmax": int(dev.argmax()),
           "dev_at": {str(i): float(dev[i]) for i in (10, 100, 500, 1000, n - 1) if i < n},
           "step1_from": a.step1_from or "fixture"}
    print(json.dumps(out), flush=True)
    if a.out:
        np.savez_compressed(a.out, losses=losses)


if __name__ == "__main__":
    main()
