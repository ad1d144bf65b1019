"""Diagnostic for the full-vs-shards linearity test (tests/test_gpu_configs.py::
test_c4_full_size_pass_per_cell_and_shared_parity): repeatability of the full pass, the
shard sum, and which bins / shards differ.  PERT_LIB selects the build under test.
usage: python tools/shard_diag.py [n_cells]"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.test_gpu_configs import _c4_full  # noqa: E402


def main():
    from scdna_replication_tools_amd.engine import EtaCodebook, PertShard
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
    sim, reads, eta, bm, t_init, libs, init = _c4_full(31, n)
    L, N = reads.shape
    common = dict(lamb=0.75, beta_means=bm, device="cuda", dirichlet_mode="exact", bins_per_tile=60)
    full = PertShard(2, reads, sim.gc, libs, 1, 13, 4, init, eta=eta, **common)
    runs = [full.loss_and_grads() for _ in range(2)]
    del full
    cuts = [(0, 2496), (2496, 4992), (4992, 7488), (7488, N)] if N == 10000 else [(0, N // 128 * 64), (N // 128 * 64, N)]
    parts, parts2 = [], []
    for i, (a, b) in enumerate(cuts):
        sl = slice(a, b)
        init_s = {k: (np.asarray(v)[sl] if k in ("expose_tau", "expose_u", "expose_betas") else v)
                  for k, v in init.items()}
        sh = PertShard(2, reads[:, sl], sim.gc, libs[sl], 1, 13, 4, init_s,
                       eta=EtaCodebook(np.ascontiguousarray(eta.codes[:, sl]), eta.table), is_root=(i == 0),
                       n_cells_total=N, **common)
        parts.append(sh.loss_and_grads())
        parts2.append(sh.loss_and_grads())
        del sh
    out = {"lib": os.environ.get("PERT_LIB", "default"), "N": N}
    for name in ("expose_rho", "expose_a", "expose_beta_stds"):
        f0 = np.asarray(runs[0][1][name], np.float64)
        f1 = np.asarray(runs[1][1][name], np.float64)
        tot = sum(np.asarray(p[1][name], np.float64) for p in parts)
        rel = np.abs(tot - f0) / np.maximum(np.abs(f0), 1e-300)
        bad = np.flatnonzero(rel > 1e-9)
        out[name] = dict(full_repeat_equal=bool(np.array_equal(f0, f1)),
                         shards_repeat_equal=[bool(np.array_equal(np.asarray(p[1][name]), np.asarray(q[1][name])))
                                              for p, q in zip(parts, parts2)],
                         n_bad=int(bad.size), max_rel=float(rel.max()) if rel.size else 0.0,
                         bad_bins=bad[:60].tolist(),
                         bad_vals=[[float(tot[j]), float(f0[j])] for j in bad[:8]])
    out["loss_rel"] = abs(sum(p[0] for p in parts) - runs[0][0]) / abs(runs[0][0])
    out["loss_full_repeat_equal"] = runs[0][0] == runs[1][0]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
