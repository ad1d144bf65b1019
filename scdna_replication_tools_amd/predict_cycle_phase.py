"""Cell-cycle phase calls from the PERT decode (reference
scdna_replication_tools/predict_cycle_phase.py:28-117), the downstream consumer of
``model_rep_state`` / ``model_cn_state``.

Same functions, arguments and output columns.  The reference loops over cells with
``groupby`` and calls ``statsmodels.tsa.acf`` per cell; here every per-cell feature is
computed at once over the cells' row segments (in each cell's row order, as ``groupby``
sees them):

* ``cell_frac_rep``: mean of the cell's replication states;
* ``rpm_auto`` / ``rep_auto``: mean of the autocorrelation function at lags 9..50
  (``np.mean(acf(x, nlags=50)[9:])``; acf is the biased estimator statsmodels returns,
  sum_t (x_t - m)(x_{t+k} - m) / sum_t (x_t - m)^2), for all lags in one pass on the
  device of the fit (or the CPU);
* ``cn_bk`` / ``rep_bk``: number of changes between consecutive rows; ``frac_cn0``.

statsmodels is not part of this stack, so the acf is restated; tests/test_phase.py pins the
batched features against a per-cell loop of that restatement.
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import pandas as pd
import torch

MIN_LAG, MAX_LAG = 10, 50


def autocorr(data, min_lag: int = MIN_LAG, max_lag: int = MAX_LAG) -> float:
    """predict_cycle_phase.py:23-25 for one series (acf restated, see module doc)."""
    x = np.asarray(data, dtype=np.float64)
    n = x.size
    d = x - x.mean()
    c0 = (d * d).sum()
    # a constant series has c0 = 0: NaN, as statsmodels' acf returns (no warning)
    with np.errstate(invalid="ignore", divide="ignore"):
        acorr = np.array([1.0] + [(d[:n - k] * d[k:]).sum() / c0 for k in range(1, max_lag + 1)])
    return float(np.mean(acorr[min_lag - 1:]))


def breakpoints(data) -> int:
    """predict_cycle_phase.py:28-30."""
    return int(np.sum(np.diff(np.asarray(data)) != 0))


def _segments(cell_ids):
    """Rows grouped by cell, each group in row order (groupby semantics): returns the sorted
    cell labels, the row permutation and the group offsets."""
    codes, cells = pd.factorize(np.asarray(cell_ids), sort=True)
    order = np.argsort(codes, kind="stable")
    counts = np.bincount(codes, minlength=len(cells))
    offs = np.concatenate([[0], np.cumsum(counts)])
    return cells, codes, order, offs


def _padded(values: np.ndarray, order, offs, device):
    """(n_cells, max_len) float64 tensor of each cell's series (zero padded) + lengths."""
    n_cells = len(offs) - 1
    lens = np.diff(offs)
    T = int(lens.max()) if n_cells else 0
    pos = np.arange(len(order)) - np.repeat(offs[:-1], lens)
    M = np.zeros((n_cells, T))
    M[np.repeat(np.arange(n_cells), lens), pos] = np.asarray(values, dtype=np.float64)[order]
    return torch.as_tensor(M, device=device), torch.as_tensor(lens, device=device)


def _batched_autocorr(M: torch.Tensor, lens: torch.Tensor, min_lag: int, max_lag: int) -> np.ndarray:
    n, T = M.shape
    idx = torch.arange(T, device=M.device)[None, :]
    valid = idx < lens[:, None]
    m = (M * valid).sum(1) / lens
    D = torch.where(valid, M - m[:, None], torch.zeros_like(M))
    c0 = (D * D).sum(1)
    ac = [torch.ones_like(c0)]
    for k in range(1, max_lag + 1):
        ac.append((D[:, :T - k] * D[:, k:]).sum(1) / c0)
    ac = torch.stack(ac, 1)
    return ac[:, min_lag - 1:].mean(1).cpu().numpy()


def compute_cell_frac(cn: pd.DataFrame, frac_rt_col='cell_frac_rep', rep_state_col='model_rep_state'):
    """predict_cycle_phase.py:33-39: per-cell fraction of replicated bins."""
    cells, codes, order, offs = _segments(cn['cell_id'].to_numpy())
    rep = cn[rep_state_col].to_numpy(np.float64)
    frac = np.bincount(codes, weights=rep, minlength=len(cells)) / np.diff(offs)
    cn[frac_rt_col] = frac[codes]
    return cn


def remove_nonreplicating_cells(cn: pd.DataFrame, frac_rt_col='cell_frac_rep', thresh=0.05):
    """predict_cycle_phase.py:42-51."""
    assert thresh < 0.5
    good_cells = cn.loc[(cn[frac_rt_col] > thresh) & (cn[frac_rt_col] < (1 - thresh))].cell_id.unique()
    keep = cn['cell_id'].isin(good_cells)
    return cn[keep].reset_index(drop=True), cn[~keep].reset_index(drop=True)


def compute_quality_features(cn: pd.DataFrame, rep_state_col='model_rep_state', cn_state_col='model_cn_state',
                             rpm_col='rpm', device: Optional[str] = None):
    """predict_cycle_phase.py:54-88: per-cell rpm / rep autocorrelation, breakpoints of the
    CN and rep calls, fraction of CN 0, and the mean-centred autocorrelations."""
    dev = torch.device(device) if device is not None else torch.device("cuda" if torch.cuda.is_available() else "cpu")
    cells, codes, order, offs = _segments(cn['cell_id'].to_numpy())
    M_rpm, lens = _padded(cn[rpm_col].to_numpy(), order, offs, dev)
    M_rep, _ = _padded(cn[rep_state_col].to_numpy(), order, offs, dev)
    rpm_auto = _batched_autocorr(M_rpm, lens, MIN_LAG, MAX_LAG)
    rep_auto = _batched_autocorr(M_rep, lens, MIN_LAG, MAX_LAG)

    def bk(col):
        v = cn[col].to_numpy()[order]
        ch = np.concatenate([[False], v[1:] != v[:-1]])
        ch[offs[:-1][np.diff(offs) > 0]] = False           # no change across a cell boundary
        return np.bincount(codes[order], weights=ch, minlength=len(cells)).astype(np.int64)

    cn0 = (cn[cn_state_col].to_numpy() == 0).astype(np.float64)
    metrics = pd.DataFrame({
        'cell_id': cells, 'rpm_auto': rpm_auto, 'rep_auto': rep_auto,
        'cn_bk': bk(cn_state_col), 'rep_bk': bk(rep_state_col),
        'frac_cn0': np.bincount(codes, weights=cn0, minlength=len(cells)) / np.diff(offs),
    })
    metrics['rpm_auto_norm'] = metrics['rpm_auto'] - np.mean(metrics['rpm_auto'].values)
    metrics['rep_auto_norm'] = metrics['rep_auto'] - np.mean(metrics['rep_auto'].values)
    # pd.merge(cn, cell_metrics): every cell has a metrics row, so the inner join keeps cn's rows
    extra = metrics.drop(columns=['cell_id']).iloc[codes].reset_index(drop=True)
    drop = [c for c in extra.columns if c in cn.columns]
    return pd.concat([cn.drop(columns=drop).reset_index(drop=True), extra], axis=1)


def remove_low_quality_cells(cn: pd.DataFrame, rep_auto_thresh=0.2, frac_cn0_thresh=0.05):
    """predict_cycle_phase.py:91-99."""
    low = cn.loc[(cn['rep_auto'] > rep_auto_thresh) | (cn['frac_cn0'] > frac_cn0_thresh)].cell_id.unique()
    bad = cn['cell_id'].isin(low)
    return cn[~bad].reset_index(drop=True), cn[bad].reset_index(drop=True)


def predict_cycle_phase(cn: pd.DataFrame, frac_rt_col='cell_frac_rep', rep_state_col='model_rep_state',
                        cn_state_col='model_cn_state', rpm_col='rpm', device: Optional[str] = None):
    """predict_cycle_phase.py:102-120: (cn_s, cn_g, cn_lq) with ``PERT_phase`` 'S' / 'G1/2' / 'LQ'."""
    cn = compute_cell_frac(cn, frac_rt_col=frac_rt_col, rep_state_col=rep_state_col)
    cn = compute_quality_features(cn, rep_state_col=rep_state_col, cn_state_col=cn_state_col, rpm_col=rpm_col,
                                  device=device)
    cn_s_lq, cn_g = remove_nonreplicating_cells(cn, frac_rt_col=frac_rt_col)
    cn_s, cn_lq = remove_low_quality_cells(cn_s_lq)
    cn_s['PERT_phase'] = 'S'
    cn_g['PERT_phase'] = 'G1/2'
    cn_lq['PERT_phase'] = 'LQ'
    return cn_s, cn_g, cn_lq
