"""Make tests/golden/c1_chain_oracle.npz: the chained fp32 oracle fit (tests/_chain.py) of the
configs[0] stand-in (tests/_configs.py: 400 S + 400 G1/2 cells x 271 bins, diploid) under
inference_tutorial.ipynb cell 9's settings (g1_clones, max_iter=200, the reference's
defaults otherwise).  The GPU test tests/test_gpu_chain.py runs the tutorial call verbatim
and compares its loss traces, decodes and final sites with this fixture.

    python tests/golden/make_chain_golden.py      (about a minute on 8 CPU threads)
"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from tests._chain import oracle_chain  # noqa: E402
from tests._configs import c1_tables, input_digest, tutorial_scrt  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "c1_chain_oracle.npz")


def main():
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    s, g, truth = c1_tables()
    digest = input_digest(s, g)
    m = tutorial_scrt(s, g, device="cpu")._pert_model()
    t0 = time.perf_counter()
    res = oracle_chain(m, torch.float32, log=lambda msg: print(msg, "{:.1f}s".format(time.perf_counter() - t0),
                                                               flush=True))
    res["input_digest"] = np.array(digest)
    res["cells_s"] = np.asarray(m._prepare().cells_s).astype("U")
    res["cells_g"] = np.asarray(m._prepare().cells_g).astype("U")
    np.savez_compressed(OUT, **res)
    print("wrote", OUT, os.path.getsize(OUT), "bytes; losses", len(res["losses_g"]), len(res["losses_s"]),
          len(res["losses_s2"]))


if __name__ == "__main__":
    main()
