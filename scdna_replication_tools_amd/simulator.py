"""Synthetic PERT data, following the reference simulator's generative model.

Reference: ``scdna_replication_tools/pert_simulator.py``
  * S-phase cells ``simulate_s_cells`` (:201-249): tau ~ Beta(1,1) (:77),
    rho = 1 - minmax(rt) (:177-179), phi = 1/(1+exp(-a (tau - rho))) (:85-88),
    rep ~ Bernoulli(phi), chi = cn (1 + rep), omega = exp(sum_k beta_k gc^(K-k)),
    u = num_reads / (1.5 L mean(cn)) (:211), delta = u chi omega (1-lam)/lam with
    delta < 1 -> 1, reads ~ NegativeBinomial(delta, probs=lam), then
    reads_norm = int64(reads / sum(reads) * num_reads) (:245-247).
  * G1/2-phase cells ``simulate_g_cells`` (:252-282): rep = 0,
    u = num_reads / (L mean(cn)).

This is a seeded numpy restatement (``numpy.random.default_rng(seed)``), used to
build the benchmark configurations and test inputs; it is
not a parity target.  NegativeBinomial(total_count=d, probs=p) is drawn as the
Gamma-Poisson mixture torch uses (Poisson(Gamma(d, scale=p/(1-p)))).
"""
from __future__ import annotations

import gzip
import io
import os
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np

_DATA = os.path.join(os.path.dirname(__file__), "data", "mcfrt.csv.gz")


def load_bins(path: str = _DATA, subdivide: int = 1):
    """The 5451 x 500 kb hg19 bin grid of the reference's ``notebooks/mcfrt.csv``
    (columns chr, start, end, gc, mcf7rt, bin_size).  ``subdivide=25`` splits every
    bin into 25 x 20 kb sub-bins that inherit the parent gc / rt (config C5)."""
    import pandas as pd
    with gzip.open(path, "rb") as fh:
        df = pd.read_csv(io.BytesIO(fh.read()), dtype={"chr": str})
    if subdivide > 1:
        size = int(df["bin_size"].iloc[0]) // subdivide
        rep = df.loc[df.index.repeat(subdivide)].reset_index(drop=True)
        k = np.tile(np.arange(subdivide), len(df))
        rep["start"] = rep["start"].values + k * size
        rep["end"] = rep["start"].values + size
        rep["bin_size"] = size
        df = rep
    return df


def convert_rt_units(rt: np.ndarray) -> np.ndarray:
    """pert_simulator.py:177-179 -- late = 1, early = 0."""
    rt = np.asarray(rt, dtype=np.float64)
    return 1 - ((rt - rt.min()) / (rt.max() - rt.min()))


def clone_profiles(n_bins: int, n_clones: int = 3) -> np.ndarray:
    """(n_bins, n_clones) somatic CN: clone A all 2; B CN 3 on bins 0-99
    (as test_with_pytest.py:21-45); C CN 1 on the last 100 bins."""
    prof = np.full((n_bins, n_clones), 2.0)
    if n_clones > 1:
        prof[: min(100, n_bins), 1] = 3.0
    if n_clones > 2:
        prof[max(0, n_bins - 100):, 2] = 1.0
    return prof


def _nb_sample(rng, total_count, probs):
    # torch.distributions.NegativeBinomial.sample: Poisson(Gamma(total_count, rate=(1-p)/p))
    rate = rng.gamma(shape=total_count, scale=probs / (1.0 - probs))
    return rng.poisson(rate).astype(np.float64)


def _gc_rate(gc, betas):
    K = len(betas) - 1
    feats = np.stack([gc ** i for i in reversed(range(K + 1))], axis=1)
    return np.exp(feats @ np.asarray(betas, dtype=np.float64))


@dataclass
class SyntheticPERT:
    """Tensor-form synthetic data: (L, N) bin-major matrices like pert_model.py:156-166."""
    gc: np.ndarray            # (L,)
    rt: np.ndarray            # (L,) raw mcf7rt
    rho_true: np.ndarray      # (L,)
    chrom: np.ndarray         # (L,)
    start: np.ndarray         # (L,)
    reads_s: np.ndarray       # (L, Ns) int64 normalised counts
    reads_g: np.ndarray       # (L, Ng)
    cn_s: np.ndarray          # (L, Ns) true somatic CN
    cn_g: np.ndarray          # (L, Ng)
    rep_s: np.ndarray         # (L, Ns) true replication state
    tau_s: np.ndarray         # (Ns,)
    clone_s: np.ndarray       # (Ns,) clone index
    clone_g: np.ndarray       # (Ng,)
    clone_cn: np.ndarray      # (L, n_clones)

    @property
    def n_bins(self):
        return self.gc.shape[0]


def simulate(n_s: int, n_g: Optional[int] = None, n_bins: Optional[int] = None, subdivide: int = 1,
             n_clones: int = 3, num_reads: float = 1e6, lamb: float = 0.75,
             betas: Sequence[float] = (0.5, 0.0), a: float = 10.0, seed: int = 0,
             bins_df=None) -> SyntheticPERT:
    """Seeded synthetic S and G1/2 cells."""
    rng = np.random.default_rng(seed)
    df = load_bins(subdivide=subdivide) if bins_df is None else bins_df
    if n_bins is not None:
        df = df.iloc[:n_bins]
    gc = df["gc"].to_numpy(np.float64)
    rt = df["mcf7rt"].to_numpy(np.float64)
    L = gc.shape[0]
    n_g = n_s if n_g is None else n_g
    prof = clone_profiles(L, n_clones)
    clone_s = np.arange(n_s) % n_clones
    clone_g = np.arange(n_g) % n_clones
    cn_s = prof[:, clone_s]
    cn_g = prof[:, clone_g]
    rho = convert_rt_units(rt)
    omega = _gc_rate(gc, betas)[:, None]

    # S-phase (pert_simulator.py:201-249)
    tau = rng.uniform(0.0, 1.0, size=n_s)
    p_rep = 1.0 / (1.0 + np.exp(-a * (tau[None, :] - rho[:, None])))
    rep = (rng.uniform(size=p_rep.shape) < p_rep).astype(np.float64)
    u_s = float(num_reads) / (1.5 * L * cn_s.mean())
    theta = u_s * cn_s * (1.0 + rep) * omega
    delta = theta * (1 - lamb) / lamb
    delta[delta < 1] = 1
    raw = _nb_sample(rng, delta, lamb)
    reads_s = (raw / raw.sum(0, keepdims=True) * num_reads).astype(np.int64)

    # G1/2-phase (pert_simulator.py:252-282)
    u_g = float(num_reads) / (1.0 * L * cn_g.mean())
    delta_g = u_g * cn_g * omega * (1 - lamb) / lamb
    delta_g[delta_g < 1] = 1
    raw_g = _nb_sample(rng, delta_g, lamb)
    reads_g = (raw_g / raw_g.sum(0, keepdims=True) * num_reads).astype(np.int64)

    return SyntheticPERT(gc=gc, rt=rt, rho_true=rho, chrom=df["chr"].to_numpy(),
                         start=df["start"].to_numpy(np.int64), reads_s=reads_s, reads_g=reads_g,
                         cn_s=cn_s, cn_g=cn_g, rep_s=rep, tau_s=tau, clone_s=clone_s,
                         clone_g=clone_g, clone_cn=prof)


def to_long_form(sim: SyntheticPERT, input_col: str = "reads", n_libs: int = 1, copy_from: str = "state",
                 order: str = "cell"):
    """Long-form DataFrames (one row per cell x bin) with the columns the
    reference entry points consume (``pert_infer_scRT``, pert_model.py:37-43) plus
    the simulator's truth columns (pert_simulator.py:371-418).

    ``copy`` (HMMcopy's copy-number estimate, the default ``assign_col``) is the true
    state (``copy_from='state'``) or a noisy estimate from the reads: each cell's reads
    scaled to its mean state (``copy_from='reads'``, what clustering needs).

    ``order='cell'``: rows grouped by cell, bins in genome order within a cell (per-cell
    HMMcopy tables concatenated, as the reference simulator's per-clone merges produce);
    ``order='bin'``: rows grouped by bin."""
    import pandas as pd
    L = sim.n_bins
    clone_names = np.array([chr(ord("A") + i) for i in range(sim.clone_cn.shape[1])], dtype=object)

    def frame(reads, cn, clone, prefix, rep=None, tau=None):
        n = reads.shape[1]
        if copy_from == "reads":
            r = reads.astype(np.float64)
            copy = r / np.maximum(r.mean(0, keepdims=True), 1e-12) * cn.mean(0, keepdims=True)
        elif copy_from == "state":
            copy = cn.astype(np.float64)
        else:
            raise ValueError(copy_from)
        # labels as object arrays: np.repeat then shares one Python string per label, as a table
        # read with pandas.read_csv holds them (its parser reuses the object of a repeated value)
        cells = np.array(["cell_{}_{}".format(prefix, i) for i in range(n)], dtype=object)
        libs = np.array(["LIB{}".format(i % n_libs) for i in range(n)], dtype=object)
        if order == "cell":
            per_bin = lambda a: np.tile(a, n)                 # (L,) bin attribute -> rows
            per_cell = lambda a: np.repeat(a, L)              # (n,) cell attribute -> rows
            flat = lambda a: np.asarray(a).T.reshape(-1)      # (L, n) matrix -> rows
        elif order == "bin":
            per_bin = lambda a: np.repeat(a, n)
            per_cell = lambda a: np.tile(a, L)
            flat = lambda a: np.asarray(a).reshape(-1)
        else:
            raise ValueError(order)
        d = {
            "cell_id": per_cell(cells),
            "chr": per_bin(sim.chrom),
            "start": per_bin(sim.start),
            "gc": per_bin(sim.gc),
            "mcf7rt": per_bin(sim.rt),
            "library_id": per_cell(libs),
            "clone_id": per_cell(clone_names[clone]),
            "state": flat(cn).astype(np.int64),
            "copy": flat(copy),
            input_col: flat(reads),
            "true_somatic_cn": flat(cn),
        }
        if rep is not None:
            d["true_rep"] = flat(rep)
            d["true_t"] = per_cell(tau)
        else:
            d["true_rep"] = np.zeros(L * n)
            d["true_t"] = np.zeros(L * n)
        return pd.DataFrame(d)

    df_s = frame(sim.reads_s, sim.cn_s, sim.clone_s, "S", sim.rep_s, sim.tau_s)
    df_g = frame(sim.reads_g, sim.cn_g, sim.clone_g, "G")
    return df_s, df_g
