"""Regenerate tests/golden/*.npz from the fp64 oracle (test infrastructure).

These fixtures pin the oracle against itself across refactors (regression) and
give the GPU suite fixed inputs; they are NOT reference outputs -- the reference
(Pyro 1.8.2) cannot be run here (parity unpinned).

    python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import pert_oracle as po  # noqa: E402
from tests._problems import make_problem  # noqa: E402


def main():
    L, N, seed = 24, 20, 13
    prob, kw, z = make_problem("step2", L=L, N=N, seed=seed)
    loss, g = po.loss_and_grads(prob, z)
    res = po.fit(prob, z, max_iter=3, min_iter=100)
    cn, rep = po.decode(prob, z)
    out = dict(L=L, N=N, seed=seed, reads=prob.reads.numpy(), loss=float(loss),
               losses3=np.array(res.losses), cn=cn.numpy().astype(np.int8), rep=rep.numpy().astype(np.int8))
    for k, v in g.items():
        out["grad_" + k] = v.numpy()
    for k, v in z.items():
        out["z_" + k] = v.numpy()
    np.savez_compressed(os.path.join(HERE, "step2_small.npz"), **out)
    print("wrote", os.path.join(HERE, "step2_small.npz"))


if __name__ == "__main__":
    main()
