"""Make tests/golden/genome_chain_oracle.npz: the chained fp32 oracle fit (tests/_chain.py,
the tensor algebra Pyro runs for pert_model.py:649-901) of a genome-length sample
(tests/_configs.py genome_tables: 64 S + 64 G1/2 cells x the full 5,451-bin 500 kb grid,
3 clones, 1e6 reads per cell, two libraries) under the reference's defaults (g1_clones
prior, max_iter 2000 / min_iter 100 / rel_tol 1e-6, steps 1 and 3 at half), with t_init
from the per-cell sklearn restatement of guess_times.  tests/test_gpu_chain.py runs
``scRT(...).infer(level='pyro')`` on the same tables and compares loss traces, stopping
iterations, decodes and final sites with this fixture.

    python tests/golden/make_genome_chain_golden.py [--chunked | --fp64]   (35-90 minutes on 8 CPU threads)
"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from tests._chain import oracle_chain  # noqa: E402
from tests._configs import genome_scrt, genome_tables, input_digest  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "genome_chain_oracle.npz")
# the same chain with the ELBO and gradients summed over 16-cell chunks: a second fp32 run of
# the same algebra whose only difference is the summation order -- how far two correct fp32
# runs drift apart over a genome-length fit (the envelope the product is held to)
OUT_CHUNKED = os.path.join(os.path.dirname(os.path.abspath(__file__)), "genome_chain_oracle_chunked.npz")
# the same chain in fp64: how far the fp32 reference's own trajectory sits from exact arithmetic
# (the product evaluates some terms more accurately than fp32 autograd)
OUT_F64 = os.path.join(os.path.dirname(os.path.abspath(__file__)), "genome_chain_oracle_f64.npz")


def main():
    chunked = "--chunked" in sys.argv
    f64 = "--fp64" in sys.argv
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    s, g, truth = genome_tables()
    digest = input_digest(s, g)
    m = genome_scrt(s, g, device="cpu")._pert_model()
    t0 = time.perf_counter()
    res = oracle_chain(m, torch.float64 if f64 else torch.float32, log=lambda msg: print(msg, "{:.1f}s".format(time.perf_counter() - t0),
                                                               flush=True), cell_chunk=16 if chunked else None)
    res["input_digest"] = np.array(digest)
    res["cells_s"] = np.asarray(m._prepare().cells_s).astype("U")
    res["cells_g"] = np.asarray(m._prepare().cells_g).astype("U")
    out = OUT_F64 if f64 else (OUT_CHUNKED if chunked else OUT)
    np.savez_compressed(out, **res)
    print("wrote", out, os.path.getsize(out), "bytes; losses", len(res["losses_g"]), len(res["losses_s"]),
          len(res["losses_s2"]))


if __name__ == "__main__":
    main()
