"""Host-side input preparation of the PERT fit, vectorised (no per-cell Python loops
over the long-form tables).

Mirrors, with identical outputs on complete inputs:
  * ``pert_infer_scRT.process_input_data`` / ``sort_by_cell_and_loci`` /
    ``get_libraries_tensor`` (reference pert_model.py:133-225)
  * ``compute_consensus_clone_profiles`` + ``add_cell_ploidies`` + ``filter_ploidies``
    (compute_consensus_clone_profiles.py:17-88)
  * the CN-prior (eta) builders ``build_cn_prior`` (:272-282), ``build_clone_cn_prior``
    (:285-296), the ``g1_cells`` branch (:671-701), ``build_composite_cn_prior`` (:299-361),
    ``diploid`` / uniform (:708-716), and ``compute_cell_corrs`` (normalize_by_cell.py:148-180)
  * ``guess_times`` / ``manhattan_binarization`` (pert_model.py:364-457)
  * ``make_g1_g2_training_data`` (:228-251)
The eta builders return an ``EtaCodebook`` (uint16 row codes + table) instead of the
dense (L, N, P) float tensor.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional

import numpy as np
import pandas as pd

from .engine import EtaCodebook

CHR_ORDER = [str(i + 1) for i in range(22)] + ["X", "Y"]


def _chr_codes(chrc: pd.Series) -> np.ndarray:
    """Chromosome category codes in CHR_ORDER (-1 for labels outside it / NaN): the
    labels are factorised first and only the few uniques go through ``str``."""
    if isinstance(chrc.dtype, pd.CategoricalDtype):
        cats = np.asarray(chrc.cat.categories)
        codes = chrc.cat.codes.to_numpy().astype(np.int64)
    else:
        codes, cats = _factorize(chrc.to_numpy())
        codes = codes.astype(np.int64)
    pos = {c: i for i, c in enumerate(CHR_ORDER)}
    lut = np.array([pos.get(str(c), -1) for c in cats] + [-1], dtype=np.int64)
    return lut[np.where(codes >= 0, codes, len(cats))]


def _object_pointers(v: np.ndarray) -> np.ndarray:
    """The PyObject addresses an object array holds, as an int64 view (no copy; valid while
    ``v`` is alive -- the caller keeps it)."""
    import ctypes
    assert v.dtype == object and v.flags.c_contiguous
    return np.ctypeslib.as_array((ctypes.c_int64 * v.size).from_address(v.ctypes.data))


def _factorize(values, sort: bool = False):
    """pd.factorize, but for object (string) columns that come in runs -- a long-form table
    grouped by cell, or by chromosome -- only the run heads are hashed: an adjacent-element
    comparison costs a fraction of hashing every Python string."""
    v = np.ascontiguousarray(values)
    if v.dtype != object or v.size < (1 << 16):
        return pd.factorize(v, sort=sort)
    probe = v[:1 << 16]
    if np.count_nonzero(probe[1:] != probe[:-1]) > probe.size // 8:
        return pd.factorize(v, sort=sort)
    # adjacent rows holding the SAME object (a label repeated by np.repeat / a per-cell
    # table concatenation) are one run: compare the object pointers first, and the values
    # (a Python comparison) only where the pointers differ
    ptr = _object_pointers(v)
    d = np.flatnonzero(ptr[1:] != ptr[:-1])
    if d.size * 4 > v.size:                           # mostly distinct objects: compare all
        d = np.flatnonzero(v[1:] != v[:-1])
    elif d.size:
        d = d[v[1:][d] != v[:-1][d]]
    heads = np.concatenate([[0], d + 1])
    if heads.size > v.size // 8:
        return pd.factorize(v, sort=sort)
    codes, uniq = pd.factorize(v[heads], sort=sort)
    return np.repeat(codes, np.diff(np.append(heads, v.size))), uniq


def _sorted_codes(values) -> tuple:
    """(codes, sorted uniques) with NaN keys coded -1, like pandas' sorted group keys."""
    codes, uniq = _factorize(values, sort=True)
    return codes.astype(np.int64), np.asarray(uniq)


def _cell_blocks(cck: np.ndarray, lkey: np.ndarray):
    """Per-cell HMMcopy tables concatenated: every cell's rows one contiguous block of L rows
    holding the SAME locus key sequence (in any order, e.g. chromosomes in file order).  The
    stable sort by (cell, chr, start) is then block order x one within-block order:
    returns the row order, or None."""
    n = cck.size
    if n == 0:
        return None
    brk = np.flatnonzero(cck[1:] != cck[:-1]) + 1
    B = brk.size + 1
    if n % B or B * 16 > n:
        return None
    L = n // B
    if brk.size and not np.array_equal(brk, np.arange(1, B) * L):
        return None
    hc = cck[::L]
    if np.unique(hc).size != B:                       # a cell split over several blocks
        return None
    k2 = lkey.reshape(B, L)
    if not (k2 == k2[:1]).all():
        return None
    q = np.argsort(k2[0], kind="stable")
    bp = np.argsort(hc, kind="stable")
    return (bp[:, None] * L + q[None, :]).reshape(-1)


def _take_columns(df: pd.DataFrame, order: np.ndarray, codes: Optional[dict] = None,
                  replace: Optional[dict] = None) -> pd.DataFrame:
    """``df.take(order)`` built column by column: numeric columns by ``np.take`` on a few
    threads (it releases the GIL), object (label) columns as ``uniques[codes[order]]`` from
    their factorisation where it is known (``codes``: (codes, uniques) by column name) -- a
    gather from a small array whose objects are shared, instead of touching one object per
    row -- and
    ``replace``: columns given directly (already in the new order)."""
    from concurrent.futures import ThreadPoolExecutor
    codes = codes or {}
    replace = replace or {}
    names = list(df.columns)
    sers = [df.iloc[:, j] for j in range(df.shape[1])]
    cols = [None] * len(sers)
    with ThreadPoolExecutor(max_workers=8) as ex:
        futs = {}
        for j, ser in enumerate(sers):
            name = names[j]
            if name in replace:
                cols[j] = replace[name]
            elif isinstance(ser.dtype, np.dtype) and ser.dtype != object:
                futs[j] = ex.submit(np.take, ser.to_numpy(), order)
            elif ser.dtype == object:
                cu = codes.get(name)
                if cu is None or len(cu[1]) * 8 > len(order):   # no codes / mostly distinct labels
                    cols[j] = np.take(ser.to_numpy(), order)
                else:
                    uext = np.empty(len(cu[1]) + 1, dtype=object)
                    uext[:-1] = cu[1]
                    uext[-1] = np.nan                     # code -1 (a missing label)
                    futs[j] = ex.submit(lambda c=cu[0], ue=uext: ue[np.take(c, order)])
            else:
                cols[j] = ser.take(order).array
        for j, f in futs.items():
            cols[j] = f.result()
    out = pd.DataFrame(dict(enumerate(cols)), index=df.index.take(order), copy=False)
    out.columns = df.columns
    return out


def _sorted_table(cn: pd.DataFrame, cell_col: str, chr_col: str, start_col: str, notna_col: Optional[str] = None):
    """``sort_by_cell_and_loci`` (pert_model.py:194-203) followed by the ``notna`` row
    filter of :139-140, as ONE take of the table, plus the integer keys of the result.
    Same stable order as ``sort_values(by=[cell, chr, start])`` (NaN keys last)."""
    cc, cells = _sorted_codes(cn[cell_col].to_numpy())
    ch = _chr_codes(cn[chr_col])
    st = cn[start_col].to_numpy()
    st_key = np.where(np.isnan(st), np.inf, st) if st.dtype.kind == "f" else st
    chk = np.where(ch < 0, len(CHR_ORDER), ch)
    cck = np.where(cc < 0, len(cells), cc)
    if st.dtype.kind in "iu" and len(st) and st.min() >= 0 and st.max() < (1 << 32) and len(cells) < (1 << 25):
        # one int64 key (cell, chr, start); a block permutation when the table comes as
        # per-cell tables with one locus order, else a stable argsort instead of a 3-key lexsort
        lkey = chk.astype(np.int64) << 32 | st.astype(np.int64)
        order = _cell_blocks(cck, lkey)
        if order is None:
            order = np.argsort(((cck.astype(np.int64) * (len(CHR_ORDER) + 1)) << 32) + lkey, kind="stable")
    else:
        order = np.lexsort((st_key, chk, cck))
    if notna_col is not None:
        ok = cn[notna_col].notna().to_numpy()
        if not ok.all():
            order = order[ok[order]]
    chr_cat = pd.Categorical.from_codes(ch[order], categories=CHR_ORDER)
    if order.size == len(cn) and (order.size == 0 or (order[1:] > order[:-1]).all()):
        out = cn.copy(deep=False)                        # already sorted and complete: no gather
        out[chr_col] = chr_cat
    else:
        out = _take_columns(cn, order, codes={cell_col: (cc, np.asarray(cells, dtype=object))},
                            replace={chr_col: chr_cat})
    return out, TableKeys.from_codes(cc[order], cells, ch[order], st[order])


def sort_by_cell_and_loci(cn: pd.DataFrame, cell_col="cell_id", chr_col="chr", start_col="start"):
    """pert_model.py:194-203: chr as a category in 1..22, X, Y order, rows sorted by
    (cell, chr, start), from integer keys (factorised cells, category codes)."""
    return _sorted_table(cn, cell_col, chr_col, start_col)[0]


@dataclass
class Pivot:
    cells: np.ndarray          # (N,) sorted cell ids (pivot_table index order)
    loci_chr: np.ndarray       # (L,) chromosome labels (category order)
    loci_start: np.ndarray     # (L,)
    values: np.ndarray         # (L, N) float64 (NaN where absent)


def _regular_rows(cell_code: np.ndarray, lkey: np.ndarray, n_cells: int) -> int:
    """L when the rows are (cell 0, loci ascending), (cell 1, the same loci), ... with every
    key valid and no locus repeated; 0 otherwise."""
    n = cell_code.size
    if n_cells == 0 or n == 0 or n % n_cells:
        return 0
    L = n // n_cells
    k0 = lkey[:L]
    if k0[0] < 0 or not (k0[1:] > k0[:-1]).all():
        return 0
    if not (cell_code.reshape(n_cells, L) == np.arange(n_cells)[:, None]).all():
        return 0
    if not (lkey.reshape(n_cells, L) == k0[None, :]).all():
        return 0
    return L


class TableKeys:
    """Integer keys of a long-form table, computed once and shared by every pivot of it:
    cell codes (sorted cell ids), locus codes (sorted (chr category, start))."""

    def __init__(self, cn: pd.DataFrame, cell_col: str, chr_col: str, start_col: str):
        cc, cells = _sorted_codes(cn[cell_col].to_numpy())
        self._set(cc, cells, _chr_codes(cn[chr_col]), cn[start_col].to_numpy())

    @classmethod
    def from_codes(cls, cell_code, cells, chr_code, start):
        k = cls.__new__(cls)
        k._set(cell_code, cells, chr_code, start)
        return k

    def _set(self, cell_code, cells, chr_code, start):
        self.cell_code, self.cells = cell_code, cells
        self.valid = (chr_code >= 0) & (cell_code >= 0)
        if start.dtype.kind == "f":
            self.valid &= ~np.isnan(start)
        lkey = np.where(self.valid, chr_code * (1 << 40) + np.where(self.valid, start, 0).astype(np.int64), -1)
        # a sorted complete table (row i = cell i // L, locus i % L, the same ascending loci in
        # every cell) needs no hashing: the locus codes are a tiled arange
        self.regular = _regular_rows(cell_code, lkey, cells.size)
        if self.regular:
            L = self.regular
            self.locus_code = np.tile(np.arange(L, dtype=np.int64), cells.size)
            ukeys = lkey[:L].copy()
        else:
            self.locus_code, ukeys = _sorted_codes(lkey)
        if ukeys.size and ukeys[0] == -1:             # drop the invalid-row key
            self.locus_code = self.locus_code - 1
            ukeys = ukeys[1:]
        cats = np.array(CHR_ORDER, dtype=object)
        self.loci_chr = cats[(ukeys >> 40).astype(int)]
        self.loci_start = ukeys & ((1 << 40) - 1)

    def _unique_positions(self, cells, loci_chr, loci_start):
        cpos = pd.Index(cells).get_indexer(self.cells)
        lidx = pd.MultiIndex.from_arrays([np.asarray(loci_chr).astype(str), np.asarray(loci_start)])
        lpos = lidx.get_indexer(pd.MultiIndex.from_arrays([self.loci_chr.astype(str), self.loci_start]))
        return cpos, lpos

    def is_grid(self, cells, loci_chr, loci_start) -> bool:
        """True when row i of the table is (cells[i // L], locus i % L) of the given axes:
        a regular table whose cells and loci are exactly the axes, in their order."""
        if not self.regular or len(cells) != self.cells.size or len(loci_start) != self.loci_start.size:
            return False
        cpos, lpos = self._unique_positions(cells, loci_chr, loci_start)
        return bool((cpos == np.arange(cpos.size)).all() and (lpos == np.arange(lpos.size)).all())

    def row_positions(self, cells, loci_chr, loci_start):
        """Per table row: the column of ``cells`` and the row of (loci_chr, loci_start) it
        belongs to (-1 where absent), via the uniques instead of per-row lookups."""
        cpos, lpos = self._unique_positions(cells, loci_chr, loci_start)
        ci = np.where(self.cell_code >= 0, cpos[np.maximum(self.cell_code, 0)], -1)
        li = np.where(self.locus_code >= 0, lpos[np.maximum(self.locus_code, 0)], -1)
        return ci, li


class RegularKeys(TableKeys):
    """TableKeys of a sorted regular table (row i = cell i // L, locus i % L, every key
    valid): the per-row code arrays are made only when a consumer asks for them."""

    def __init__(self, cells, loci_chr, loci_start, L: int):
        self.cells = np.asarray(cells)
        self.loci_chr = np.asarray(loci_chr, dtype=object)
        self.loci_start = np.asarray(loci_start)
        self.regular = int(L)
        self._cc = self._lc = None

    @property
    def n_rows(self) -> int:
        return self.cells.size * self.regular

    @property
    def cell_code(self):
        if self._cc is None:
            self._cc = np.repeat(np.arange(self.cells.size, dtype=np.int64), self.regular)
        return self._cc

    @property
    def locus_code(self):
        if self._lc is None:
            self._lc = np.tile(np.arange(self.regular, dtype=np.int64), self.cells.size)
        return self._lc

    @property
    def valid(self):
        return np.ones(self.n_rows, dtype=bool)


def _n_rows(keys) -> int:
    return keys.n_rows if isinstance(keys, RegularKeys) else len(keys.cell_code)


def _same_objects(a: np.ndarray, B: int, L: int) -> bool:
    """Every (B, L) row of the object column ``a`` holds the values of its first row: by
    object identity first, values compared only where the objects differ."""
    a = np.ascontiguousarray(a)
    if a.dtype != object:
        a2 = a.reshape(B, L)
        return bool((a2 == a2[:1]).all())
    p2 = _object_pointers(a).reshape(B, L)
    diff = p2 != p2[:1]
    if not diff.any():
        return True
    if diff.sum() * 16 > a.size:
        return False                                   # mostly distinct objects: the general path
    a2 = a.reshape(B, L)
    return bool((a2[diff] == np.broadcast_to(a2[:1], (B, L))[diff]).all())


def _constant_rows(a: np.ndarray, B: int, L: int) -> bool:
    """Every (B, L) row of ``a`` holds one value (object identity first, as _same_objects)."""
    a = np.ascontiguousarray(a)
    if a.dtype != object:
        a2 = a.reshape(B, L)
        return bool((a2 == a2[:, :1]).all())
    p2 = _object_pointers(a).reshape(B, L)
    diff = p2 != p2[:, :1]
    if not diff.any():
        return True
    if diff.sum() * 16 > a.size:
        return False
    a2 = a.reshape(B, L)
    return bool((a2[diff] == np.broadcast_to(a2[:, :1], (B, L))[diff]).all())


def _block_layout(cn: pd.DataFrame, cell_col: str, chr_col: str, start_col: str, notna_col: Optional[str]):
    """Per-cell blocks (the per-cell HMMcopy tables concatenated): every cell's rows one
    contiguous block of L rows, every block the same valid locus sequence (any order, no
    repeats).  Found from the block heads only -- object identity runs of the cell column, one
    integer compare of the starts, one identity compare of the chromosome labels -- without
    hashing any per-row string.  Returns (B, L, bp, q, chr codes of block 0) with ``bp`` the
    blocks in sorted cell order and ``q`` the loci of a block in (chr, start) order, or None."""
    cell = np.ascontiguousarray(cn[cell_col].to_numpy())
    n = cell.size
    if n == 0 or cell.dtype != object:
        return None
    ptr = _object_pointers(cell)
    d = np.flatnonzero(ptr[1:] != ptr[:-1])
    if d.size * 16 > n:
        return None
    if d.size:
        d = d[cell[1:][d] != cell[:-1][d]]
    B = d.size + 1
    if n % B or B * 16 > n:
        return None
    L = n // B
    if B > 1 and not np.array_equal(d + 1, np.arange(1, B, dtype=d.dtype) * L):
        return None
    names = cell[::L]
    if not all(isinstance(x, str) for x in names) or len(set(names)) != B:
        return None
    st = cn[start_col].to_numpy()
    if st.dtype.kind not in "iu" or (st.size and (st.min() < 0 or st.max() >= (1 << 32))):
        return None
    if not _same_objects(st, B, L):
        return None
    chc = cn[chr_col]
    if isinstance(chc.dtype, pd.CategoricalDtype):
        if not _same_objects(chc.cat.codes.to_numpy(), B, L):
            return None
    elif not _same_objects(chc.to_numpy(), B, L):
        return None
    ch0 = _chr_codes(chc.iloc[:L])
    if (ch0 < 0).any():
        return None
    if notna_col is not None:
        v = cn[notna_col].to_numpy()
        if v.dtype.kind == "f" and np.isnan(v).any():
            return None
        if v.dtype == object and pd.isna(v).any():
            return None
    lkey0 = ch0.astype(np.int64) << 32 | st[:L].astype(np.int64)
    q = np.argsort(lkey0, kind="stable")
    if np.unique(lkey0).size != L:
        return None                                    # a locus twice in a cell: the general path
    bp = np.argsort(names, kind="stable")
    return B, L, bp, q, ch0


def pivot_cells_by_loci(cn: pd.DataFrame, value_col: str, cell_col: str, chr_col: str, start_col: str,
                        keys: Optional[TableKeys] = None) -> Pivot:
    """``cn.pivot_table(index=cell, columns=[chr, start], values=col).T`` without the
    pandas machinery: sorted cells, loci in (chromosome category, start) order,
    duplicates averaged (pivot_table's default aggfunc), rows with a NaN key or value
    dropped, cells / loci with no value at all dropped (pivot_table's dropna)."""
    k = TableKeys(cn, cell_col, chr_col, start_col) if keys is None else keys
    val = cn[value_col].to_numpy(np.float64)
    if getattr(k, "regular", 0) and val.size == _n_rows(k):
        # one row per (cell, locus) in (cell, locus) order: the pivot is a transpose
        N, L = k.cells.size, k.loci_start.size
        out = np.ascontiguousarray(val.reshape(N, L).T)
        nan = np.isnan(out)
        if nan.any():
            has_l, has_c = ~nan.all(axis=1), ~nan.all(axis=0)
            if not (has_l.all() and has_c.all()):
                return Pivot(k.cells[has_c], k.loci_chr[has_l], k.loci_start[has_l], out[has_l][:, has_c])
        return Pivot(k.cells, k.loci_chr, k.loci_start, out)
    keep = k.valid & ~np.isnan(val)
    ci, li = k.cell_code[keep], k.locus_code[keep]
    N, L = k.cells.size, k.loci_start.size
    lin = li * N + ci
    s = np.bincount(lin, weights=val[keep], minlength=L * N).reshape(L, N)
    c = np.bincount(lin, minlength=L * N).reshape(L, N)
    with np.errstate(invalid="ignore", divide="ignore"):
        out = np.where(c > 0, s / np.maximum(c, 1), np.nan)
    has_l = c.any(axis=1)
    has_c = c.any(axis=0)
    if not (has_l.all() and has_c.all()):
        out = out[has_l][:, has_c]
        return Pivot(k.cells[has_c], k.loci_chr[has_l], k.loci_start[has_l], out)
    return Pivot(k.cells, k.loci_chr, k.loci_start, out)


def drop_incomplete_loci(p: Pivot) -> Pivot:
    """``.dropna(axis=1)`` on the (cell x locus) pivot (pert_model.py:148-151)."""
    ok = ~np.isnan(p.values).any(axis=1)
    return Pivot(p.cells, p.loci_chr[ok], p.loci_start[ok], p.values[ok])


@dataclass
class PertInputs:
    """Tensor inputs of the three fits (pert_model.py:191)."""
    loci_chr: np.ndarray
    loci_start: np.ndarray
    cells_s: np.ndarray
    cells_g: np.ndarray
    reads_s: np.ndarray        # (L, Ns) float32 (int64-truncated, :163-166)
    states_s: np.ndarray       # (L, Ns) float32
    reads_g: np.ndarray        # (L, Ng)
    states_g: np.ndarray
    gc: np.ndarray             # (L,) float32
    libs_s: np.ndarray         # (Ns,) int64
    libs_g: np.ndarray
    library_ids: list
    keys_s: Optional["TableKeys"] = None      # integer keys of the sorted long tables (row order)
    keys_g: Optional["TableKeys"] = None
    # the input_col pivots before the int64 truncation of :163-166, kept only when the input
    # is not integer valued: the eta builders correlate the long table's raw values
    reads_s_raw: Optional[np.ndarray] = None
    reads_g_raw: Optional[np.ndarray] = None


def _trunc32(a):
    a = np.asarray(a)
    if a.dtype == np.float32:
        return a                   # a block pivot of an integer column: already the exact values
    return a.astype(np.int64).astype(np.float32)


def _align(p: Pivot, chr_, start) -> Pivot:
    if (len(p.loci_start) == len(start) and np.array_equal(p.loci_start, start)
            and np.array_equal(np.asarray(p.loci_chr).astype(str), np.asarray(chr_).astype(str))):
        return p                                        # already in that locus order
    key = pd.MultiIndex.from_arrays([p.loci_chr, p.loci_start])
    want = pd.MultiIndex.from_arrays([chr_, start])
    idx = key.get_indexer(want)
    assert (idx >= 0).all()
    return Pivot(p.cells, p.loci_chr[idx], p.loci_start[idx], p.values[idx])


def _cell_libraries(cn: pd.DataFrame, keys: TableKeys, library_col: str, cells: np.ndarray):
    """(cell, library) pairs of get_libraries_tensor (:206-225) from the integer keys:
    the library labels in first-appearance order and one label per pivot cell."""
    if isinstance(keys, RegularKeys) and isinstance(cn, DeferredTable):
        # the source's blocks (constant within a block in any row order), heads in sorted order
        B, L = keys.cells.size, keys.regular
        v = cn.source[library_col].to_numpy()
        if v.size == B * L and _constant_rows(v, B, L):
            per_cell = cn.column_at(library_col, np.arange(B, dtype=np.int64) * L)
            if not pd.isna(per_cell).any():
                ids = list(pd.unique(per_cell))          # first appearance over the sorted rows
                lab = pd.Series(per_cell, index=pd.Index(keys.cells)).reindex(np.asarray(cells)).to_numpy()
                return ids, lab
        cn = cn.result()
    if isinstance(keys, RegularKeys):
        # one label per cell block (else the general path below finds and refuses the cell
        # with two libraries)
        v = cn[library_col].to_numpy()
        B, L = keys.cells.size, keys.regular
        if v.size == B * L and _constant_rows(v, B, L):
            per_cell = v[::L]                            # one label per sorted cell
            if not pd.isna(per_cell).any():
                ids = list(pd.unique(per_cell))          # first appearance over the sorted rows
                lab = pd.Series(per_cell, index=pd.Index(keys.cells)).reindex(np.asarray(cells)).to_numpy()
                return ids, lab
    lib_code, lib_uniq = _factorize(cn[library_col].to_numpy())
    cc = keys.cell_code
    fast = False
    if getattr(keys, "regular", 0) and lib_code.size == cc.size:
        # regular table: cell c is rows [c L, (c+1) L); one library per cell is a row compare
        lc2 = np.asarray(lib_code).reshape(keys.cells.size, keys.regular)
        if (lc2[:, 0] >= 0).all():
            if not (lc2 == lc2[:, :1]).all():
                raise ValueError("a cell belongs to more than one {}".format(library_col))
            pl = lc2[:, 0].astype(np.int64)
            per_cell = pl
            fast = True
    if not fast:
        ok = cc >= 0
        pairs = pd.unique(cc[ok] * (len(lib_uniq) + 1) + lib_code[ok])
        pc, pl = pairs // (len(lib_uniq) + 1), pairs % (len(lib_uniq) + 1)
        if np.unique(pc).size != pc.size:
            raise ValueError("a cell belongs to more than one {}".format(library_col))
        per_cell = np.full(keys.cells.size, -1, np.int64)
        per_cell[pc] = pl
    order = pd.unique(pl)                                # first appearance over the (sorted) rows
    sel = pd.Index(keys.cells).get_indexer(cells)
    return [lib_uniq[i] for i in order], lib_uniq[per_cell[sel]]


def process_input_data(cn_s: pd.DataFrame, cn_g1: pd.DataFrame, input_col="reads", gc_col="gc",
                       cell_col="cell_id", library_col="library_id", chr_col="chr", start_col="start",
                       cn_state_col="state", on_g1_sorted=None, defer_sorted: bool = False):
    """pert_model.py:133-191 (the unused rt prior aside).  Returns the sorted,
    NaN-filtered long tables and a ``PertInputs``.  ``on_g1_sorted(table, keys)`` is called
    with the sorted G1/2 table as soon as it exists (work that needs only it can start while
    the S table is still being prepared).  ``defer_sorted``: a per-cell-block table's sorted
    copy comes back as a DeferredTable built on a background thread (the pivots, keys, library
    index and gc are made without it)."""
    from concurrent.futures import ThreadPoolExecutor

    def table(cn, hook=None):
        # the two tables are independent: sorted and pivoted on two threads (the numpy
        # passes release the GIL; the object-column passes interleave)
        lay = _block_layout(cn, cell_col, chr_col, start_col, input_col)
        if lay is not None:
            return _block_table(cn, lay, hook, input_col, cn_state_col, cell_col, chr_col, start_col,
                                defer=defer_sorted)
        cn, k = _sorted_table(cn, cell_col, chr_col, start_col, notna_col=input_col)
        if hook is not None:
            hook(cn, k)
        r = drop_incomplete_loci(pivot_cells_by_loci(cn, input_col, cell_col, chr_col, start_col, k))
        st = drop_incomplete_loci(pivot_cells_by_loci(cn, cn_state_col, cell_col, chr_col, start_col, k))
        return cn, k, r, st

    with ThreadPoolExecutor(max_workers=2) as ex:
        fg, fs = ex.submit(table, cn_g1, on_g1_sorted), ex.submit(table, cn_s)
        cn_g1, kg, pg_r, pg_s = fg.result()
        cn_s, ks, ps_r, ps_s = fs.result()
    assert pg_s.values.shape == pg_r.values.shape                      # :153
    assert ps_r.values.shape[0] == pg_r.values.shape[0]                 # :154
    ps_s = _align(ps_s, ps_r.loci_chr, ps_r.loci_start) if ps_s.values.shape == ps_r.values.shape else ps_s
    pg_s = _align(pg_s, pg_r.loci_chr, pg_r.loci_start)

    # library index: first appearance over S then G1 cells (get_libraries_tensor, :206-225)
    ids_s, lab_s = _cell_libraries(cn_s, ks, library_col, ps_r.cells)
    ids_g, lab_g = _cell_libraries(cn_g1, kg, library_col, pg_r.cells)
    all_ids = list(pd.unique(np.asarray(ids_s + ids_g, dtype=object)))
    lut = {v: i for i, v in enumerate(all_ids)}
    libs_s = np.array([lut[v] for v in lab_s], np.int64)
    libs_g = np.array([lut[v] for v in lab_g], np.int64)
    assert libs_s.shape[0] == ps_r.values.shape[1] and libs_g.shape[0] == pg_r.values.shape[1]

    # gc per locus: first row of each locus in the sorted S table
    if isinstance(cn_s, DeferredTable):
        gc_locus = cn_s.column_at(gc_col, np.arange(ks.regular)).astype(np.float64)   # cell 0's rows
        gcv = None
    else:
        gcv = cn_s[gc_col].to_numpy(np.float64)
    if gcv is None:
        pass
    elif getattr(ks, "regular", 0) and gcv.size == _n_rows(ks):
        gc_locus = gcv[:ks.regular]                      # regular table: cell 0's rows, locus order
    else:
        okr = ks.valid
        _, first = np.unique(ks.locus_code[okr], return_index=True)
        gc_locus = gcv[np.flatnonzero(okr)[first]]
    gkey = pd.MultiIndex.from_arrays([ks.loci_chr.astype(str), ks.loci_start])
    gi = gkey.get_indexer(pd.MultiIndex.from_arrays([ps_r.loci_chr.astype(str), ps_r.loci_start]))
    gc = gc_locus[gi].astype(np.float32)
    if np.isnan(gc).any():
        raise ValueError("{} is missing for some loci".format(gc_col))

    reads_s, reads_g = _trunc32(ps_r.values), _trunc32(pg_r.values)
    raw = lambda v, t: None if (v is t or np.array_equal(v, t)) else v
    inp = PertInputs(loci_chr=ps_r.loci_chr, loci_start=ps_r.loci_start, cells_s=ps_r.cells, cells_g=pg_r.cells,
                     reads_s=reads_s, states_s=_trunc32(ps_s.values),
                     reads_g=reads_g, states_g=_trunc32(pg_s.values), gc=gc,
                     libs_s=libs_s, libs_g=libs_g, library_ids=all_ids, keys_s=ks, keys_g=kg,
                     reads_s_raw=raw(ps_r.values, reads_s), reads_g_raw=raw(pg_r.values, reads_g))
    return cn_s, cn_g1, inp


def _block_pivot(v: np.ndarray, B: int, L: int, bp: np.ndarray, q: np.ndarray) -> np.ndarray:
    """The (loci x cells) pivot of a per-cell-block column: (L, B), cells in sorted order
    (``bp``), loci in (chr, start) order (``q``) -- a transpose of the blocks.  Integer
    columns whose values fp32 holds exactly come as float32 (the int64-truncated fp32 tensor
    of pert_model.py:163-166 itself), others as float64."""
    from concurrent.futures import ThreadPoolExecutor
    g = np.asarray(v).reshape(B, L)
    same_b, same_q = np.array_equal(bp, np.arange(B)), np.array_equal(q, np.arange(L))
    # cell tiles on a few threads (numpy's gathers, reductions and casting copies release the
    # GIL): one gather + transpose + cast per tile, instead of a strided whole-matrix copy
    T = 64
    starts = range(0, B, T)
    with ThreadPoolExecutor(max_workers=8) as ex:
        exact32 = g.dtype.kind in "iu"
        if exact32 and g.size:
            mm = list(ex.map(lambda j0: (g[j0:j0 + 4 * T].min(), g[j0:j0 + 4 * T].max()), range(0, B, 4 * T)))
            exact32 = min(m[0] for m in mm) > -(1 << 24) and max(m[1] for m in mm) < (1 << 24)
        out = np.empty((L, B), dtype=np.float32 if exact32 else np.float64)

        def tile(j0):
            j1 = min(B, j0 + T)
            t = g[j0:j1] if same_b else g[bp[j0:j1]]
            out[:, j0:j1] = (t if same_q else t[:, q]).T
        list(ex.map(tile, starts))
    return out


def transpose_cast(a: np.ndarray, dtype) -> np.ndarray:
    """``np.ascontiguousarray(a.T).astype(dtype)`` for a (loci x cells) matrix: the (cells x
    loci) rows a long table in (cell, locus) order holds, by cell tiles on a few threads (one
    transpose + cast per tile, as _block_pivot)."""
    from concurrent.futures import ThreadPoolExecutor
    a = np.asarray(a)
    L, N = a.shape
    out = np.empty((N, L), dtype=dtype)
    T = 64

    def tile(j0):
        out[j0:j0 + T] = a[:, j0:j0 + T].T
    with ThreadPoolExecutor(max_workers=8) as ex:
        list(ex.map(tile, range(0, N, T)))
    return out


def pivot_any(cn: pd.DataFrame, value_col: str, cell_col: str, chr_col: str, start_col: str) -> Pivot:
    """pivot_cells_by_loci, through the block transpose when the table is per-cell blocks with no
    missing value (the same sorted cells, loci and values), else the general path."""
    lay = _block_layout(cn, cell_col, chr_col, start_col, value_col)
    if lay is None:
        return pivot_cells_by_loci(cn, value_col, cell_col, chr_col, start_col)
    B, L, bp, q, ch0 = lay
    cells = np.ascontiguousarray(cn[cell_col].to_numpy())[::L][bp]
    vals = _block_pivot(cn[value_col].to_numpy(), B, L, bp, q).astype(np.float64, copy=False)
    return Pivot(cells, np.array(CHR_ORDER, dtype=object)[ch0[q]], cn[start_col].to_numpy()[:L][q], vals)


_DEFER_POOL = None
_DEFER_LOCK = __import__("threading").Lock()


def _defer_pool():
    global _DEFER_POOL
    with _DEFER_LOCK:
        if _DEFER_POOL is None:
            from concurrent.futures import ThreadPoolExecutor
            _DEFER_POOL = ThreadPoolExecutor(max_workers=2, thread_name_prefix="pert-sort")
        return _DEFER_POOL


class DeferredTable:
    """The sorted copy of a per-cell-block table (sort_by_cell_and_loci, pert_model.py:194-203),
    built on a background thread once ``start()`` is called (or on first ``result()``): the fit
    needs only the pivots to start, packaging needs the copy seconds later.  ``result()`` waits for it; ``column_at(name, rows)`` reads a column at
    rows of the sorted order straight from the source table (sorted row r is the source's row
    bp[r // L] L + q[r % L]), so the per-cell labels the priors and the library index take from
    a cell's first row need no copy."""

    def __init__(self, source: pd.DataFrame, lay, build):
        self.source = source
        self.lay = lay
        self._build = build
        self._fut = None
        self._lock = __import__("threading").Lock()

    def start(self) -> "DeferredTable":
        """Begin the copy on the background thread (a fit starts it once its own host work is
        done: the copy's object columns hold the interpreter lock for much of their time)."""
        with self._lock:
            if self._fut is None:
                self._fut = _defer_pool().submit(self._build)
        return self

    def __len__(self) -> int:
        return self.lay[0] * self.lay[1]

    def result(self) -> pd.DataFrame:
        return self.start()._fut.result()

    def column_at(self, name: str, rows: np.ndarray) -> np.ndarray:
        B, L, bp, q, _ = self.lay
        rows = np.asarray(rows, dtype=np.int64)
        return self.source[name].to_numpy()[bp[rows // L].astype(np.int64) * L + q[rows % L]]


def resolved(cn):
    """The table itself (a DeferredTable's sorted copy, once built)."""
    return cn.result() if isinstance(cn, DeferredTable) else cn


def _block_table(cn, lay, hook, input_col, cn_state_col, cell_col, chr_col, start_col, defer: bool = False):
    """process_input_data's per-table work for a per-cell-block table (_block_layout): the
    table sorted by (cell, chr, start) with one gather per column (the cell and chromosome
    columns rebuilt from the block heads), RegularKeys, and the two pivots as transposes of
    the blocks -- no per-row hashing of the labels."""
    B, L, bp, q, ch0 = lay
    cells = np.ascontiguousarray(cn[cell_col].to_numpy())[::L][bp]
    chq = ch0[q]
    loci_chr = np.array(CHR_ORDER, dtype=object)[chq]
    loci_start = cn[start_col].to_numpy()[:L][q]

    def build():
        order = (bp.astype(np.int64)[:, None] * L + q[None, :]).reshape(-1)
        chr_cat = pd.Categorical.from_codes(np.tile(chq.astype(np.int8), B), categories=CHR_ORDER)
        replace = {cell_col: np.repeat(cells.astype(object), L), chr_col: chr_cat}
        for name in cn.columns:
            # per-cell label columns (library, clone): one object per block, by identity -- the
            # block heads repeated instead of a gather of every row
            if name in replace or name == cell_col or cn[name].dtype != object:
                continue
            a = np.ascontiguousarray(cn[name].to_numpy())
            p2 = _object_pointers(a).reshape(B, L)
            if (p2 == p2[:, :1]).all():
                replace[name] = np.repeat(a[::L][bp], L)
        return _take_columns(cn, order, replace=replace)
    out = DeferredTable(cn, lay, build) if defer else build()
    k = RegularKeys(cells, loci_chr, loci_start, L)
    if hook is not None:
        hook(out, k)

    def pivot(col):
        v = cn[col].to_numpy()
        if v.dtype.kind == "f" and np.isnan(v).any():
            # missing values: pivot_table's NaN handling on the sorted table
            return drop_incomplete_loci(pivot_cells_by_loci(resolved(out), col, cell_col, chr_col, start_col, k))
        return Pivot(cells, loci_chr, loci_start, _block_pivot(v, B, L, bp, q))
    return out, k, pivot(input_col), pivot(cn_state_col)


# --------------------------------------------------------------------------- clones
def _factorize_sorted_numbers(values):
    """pd.factorize(values, sort=True) for a numeric column; small non-negative integers
    (CN states) by one bincount instead of hashing every row."""
    v = np.asarray(values)
    if v.size and v.dtype.kind in "iuf":
        lo, hi = v.min(), v.max()                       # NaN propagates: no fast path
        if lo >= 0 and hi < 4096 and (v.dtype.kind in "iu" or (v == np.floor(v)).all()):
            vi = v.astype(np.int64)
            present = np.bincount(vi, minlength=int(hi) + 1) > 0
            remap = np.cumsum(present) - 1
            return remap[vi], np.flatnonzero(present).astype(v.dtype)
    return pd.factorize(v, sort=True)


def _cell_mode(cell_code: np.ndarray, n_cells: int, states: np.ndarray) -> np.ndarray:
    """Per-cell mode of ``states`` (ties to the smallest value, scipy.stats.mode), by
    counting (cell, state) codes."""
    sc, su = _factorize_sorted_numbers(states)
    ok = (sc >= 0) & (cell_code >= 0)
    cnt = np.bincount(cell_code[ok] * len(su) + sc[ok], minlength=n_cells * len(su)).reshape(n_cells, len(su))
    return np.asarray(su)[cnt.argmax(axis=1)] if len(su) else np.full(n_cells, np.nan)


def cell_ploidies(cn: pd.DataFrame, cell_col="cell_id", cn_state_col="state") -> pd.Series:
    """add_cell_ploidies (compute_consensus_clone_profiles.py:30-39): per-cell mode of the
    CN state, ties to the smallest value (scipy.stats.mode)."""
    cc, cells = _sorted_codes(cn[cell_col].to_numpy())
    return pd.Series(_cell_mode(cc, len(cells), cn[cn_state_col].to_numpy()), index=pd.Index(cells, name=cell_col),
                     name=cn_state_col)


def _majority_ploidy_rows(cn: pd.DataFrame, clone_col="clone_id", cell_col="cell_id", cn_state_col="state",
                          cell_code=None, n_cells=None, clone_code=None, n_clones=None):
    """Row mask of add_cell_ploidies + filter_ploidies (:17-39): each cell's ploidy is the
    mode of its states; each clone keeps the rows of its most frequent ploidy (row counts,
    ties to the smallest ploidy, ``idxmax`` over the sorted ploidy index)."""
    if cell_code is None:
        cell_code, cells = _sorted_codes(cn[cell_col].to_numpy())
        n_cells = len(cells)
    if clone_code is None:
        clone_code, ku = _factorize(cn[clone_col].to_numpy())
        n_clones = len(ku)
    cc, kc = cell_code, clone_code
    pl_cell = _cell_mode(cc, n_cells, cn[cn_state_col].to_numpy())
    # ploidy codes per cell, then per row (the per-cell uniques may include ploidies of cells
    # without rows here: they only add zero-count columns, which no argmax below picks)
    pcc, pu = pd.factorize(pl_cell, sort=True)
    pc = pcc[np.where(cc >= 0, cc, 0)]
    ok = (kc >= 0) & (pc >= 0) & (cc >= 0)
    cnt = np.bincount(kc[ok] * len(pu) + pc[ok], minlength=n_clones * len(pu)).reshape(n_clones, len(pu))
    keep_pc = cnt.argmax(axis=1)
    return ok & (pc == keep_pc[np.where(kc >= 0, kc, 0)])


def filter_ploidies(cn: pd.DataFrame, ploidy: Optional[pd.Series] = None, clone_col="clone_id", cell_col="cell_id",
                    cn_state_col="state", ploidy_col: Optional[str] = None):
    """filter_ploidies (:17-27): keep the rows of the majority ploidy of each clone (row
    counts, ties to the smallest ploidy; rows of a NaN clone or NaN ploidy dropped).  The
    per-row ploidy is ``cn[ploidy_col]`` when given, else ``ploidy`` mapped per cell, else
    each cell's modal state (add_cell_ploidies, :30-39)."""
    if ploidy_col is not None:
        pl = cn[ploidy_col].to_numpy()
    elif ploidy is None:
        return cn[_majority_ploidy_rows(cn, clone_col, cell_col, cn_state_col)]
    else:
        pl = cn[cell_col].map(ploidy).to_numpy()
    kc, ku = _factorize(cn[clone_col].to_numpy())
    pc, pu = pd.factorize(pl, sort=True)
    ok = (kc >= 0) & (pc >= 0)
    cnt = np.bincount(kc[ok] * len(pu) + pc[ok], minlength=len(ku) * len(pu)).reshape(len(ku), len(pu))
    return cn[ok & (pc == cnt.argmax(axis=1)[np.where(kc >= 0, kc, 0)])]


def _group_median_small_ints(g: np.ndarray, v: np.ndarray, n_groups: int, n_vals: int) -> np.ndarray:
    """Per-group median of small non-negative integers (CN states) from a (group, value)
    histogram: the order statistics lo = (n-1)//2 and hi = n//2 are read off the cumulative
    counts -- the values the sort below would pick, without sorting."""
    cnt = np.bincount(g * n_vals + v, minlength=n_groups * n_vals).reshape(n_groups, n_vals)
    cum = np.cumsum(cnt, axis=1)
    n = cum[:, -1]
    out = np.full(n_groups, np.nan)
    has = n > 0
    c, nh = cum[has], n[has]
    lo = (c <= ((nh - 1) // 2)[:, None]).sum(axis=1)     # first value whose cumulative count passes lo
    hi = (c <= (nh // 2)[:, None]).sum(axis=1)
    out[has] = 0.5 * (lo + hi)
    return out


def _group_median(group: np.ndarray, values: np.ndarray, n_groups: int) -> np.ndarray:
    """Median of ``values`` per group code (NaN for empty groups), by one lexsort."""
    ok = ~np.isnan(values) & (group >= 0)
    g, v = group[ok], values[ok]
    if v.size and n_groups * 64 <= max(v.size, 1 << 20):
        lo_v, hi_v = v.min(), v.max()
        if lo_v >= 0 and hi_v < 64 and (v == np.floor(v)).all():
            return _group_median_small_ints(g, v.astype(np.int64), n_groups, int(hi_v) + 1)
    order = np.lexsort((v, g))
    g, v = g[order], v[order]
    n = np.bincount(g, minlength=n_groups)
    first = np.concatenate([[0], np.cumsum(n)[:-1]])
    out = np.full(n_groups, np.nan)
    has = n > 0
    lo = first[has] + (n[has] - 1) // 2
    hi = first[has] + n[has] // 2
    out[has] = 0.5 * (v[lo] + v[hi])
    return out


def _consensus_blocks(cn: pd.DataFrame, col_name: str, clone_col: str, cn_state_col, keys: "RegularKeys"):
    """consensus_clone_profiles' medians on a regular sorted table (every cell one block of
    the same L loci, one clone per cell): ``consensus_arrays`` on its columns.  (L,
    n_clones) and the sorted clone ids, or None (the general path)."""
    B, L = keys.cells.size, keys.regular
    return consensus_arrays(cn[clone_col].to_numpy(), cn[col_name].to_numpy(np.float64),
                            None if cn_state_col is None else cn[cn_state_col].to_numpy(), B, L)


def consensus_arrays(clone: np.ndarray, values: np.ndarray, states: Optional[np.ndarray], B: int, L: int):
    """The medians of compute_consensus_clone_profiles (:42-88) for a table of B per-cell
    blocks of the same L loci (rows b L .. b L + L - 1 are cell b's, in one locus order): each
    cell's modal state, each clone's majority ploidy (row counts are L per cell, so cell counts
    decide), and per clone a column median over its kept cells.  Neither the order of the cells
    nor that of the loci matters (medians and counts); rows come out in the blocks' locus order.
    (L, n_clones) and the sorted clone ids, or None (NaN values or states, a cell in two
    clones: the general path)."""
    if clone.size != B * L or not _constant_rows(clone, B, L):
        return None
    kcell, ku = _sorted_codes(clone[::L])
    if "None" in set(ku.tolist()):                       # clone 'None' is removed (:63)
        bad = int(np.flatnonzero(ku == "None")[0])
        kcell = np.where(kcell == bad, -1, kcell)
    vals = np.asarray(values, dtype=np.float64).reshape(B, L)
    if np.isnan(vals).any():
        return None
    keep = kcell >= 0
    if states is not None:
        st = np.asarray(states).reshape(B, L)
        if st.dtype.kind not in "iu":
            if st.dtype.kind != "f" or np.isnan(st).any() or not (st == np.floor(st)).all():
                return None
        lo, hi = int(st.min()), int(st.max())
        if lo < 0 or hi >= 4096:
            return None
        cnt = _row_state_counts(st, hi + 1)
        pl = cnt.argmax(axis=1)                          # modal state, ties to the smallest
        pu = np.unique(pl)
        pc = np.searchsorted(pu, pl)
        cc = np.bincount(kcell[keep] * len(pu) + pc[keep], minlength=len(ku) * len(pu)).reshape(len(ku), len(pu))
        keep &= pc == cc.argmax(axis=1)[np.where(kcell >= 0, kcell, 0)]
    med = np.full((L, len(ku)), np.nan)
    for c in range(len(ku)):
        rows = np.flatnonzero(keep & (kcell == c))
        if rows.size:
            med[:, c] = _column_median(vals, rows)
    return med, ku


def _row_state_counts(st: np.ndarray, n_vals: int) -> np.ndarray:
    """(B, n_vals) counts of each state in each row of the integer-valued (B, L) ``st``
    (values in [0, n_vals)): one bincount per tile of rows, tiles on a few threads."""
    from concurrent.futures import ThreadPoolExecutor
    B = st.shape[0]
    out = np.empty((B, n_vals), np.int64)
    T = 256

    def tile(b0):
        s = st[b0:b0 + T].astype(np.int64)
        n = s.shape[0]
        out[b0:b0 + n] = np.bincount((np.arange(n, dtype=np.int64)[:, None] * n_vals + s).reshape(-1),
                                     minlength=n * n_vals).reshape(n, n_vals)
    with ThreadPoolExecutor(max_workers=8) as ex:
        list(ex.map(tile, range(0, B, T)))
    return out


def _column_median(vals: np.ndarray, rows: np.ndarray) -> np.ndarray:
    """np.median(vals[rows], axis=0) for a (cells, L) matrix: locus tiles on a few threads,
    each gathered and transposed so the median runs along contiguous rows (np.median of the
    same values per locus: the same result)."""
    from concurrent.futures import ThreadPoolExecutor
    L = vals.shape[1]
    out = np.empty(L)
    T = 256

    def tile(l0):
        out[l0:l0 + T] = np.median(np.ascontiguousarray(vals[rows, l0:l0 + T].T), axis=1)
    with ThreadPoolExecutor(max_workers=8) as ex:
        list(ex.map(tile, range(0, L, T)))
    return out


def consensus_from_blocks(cn: pd.DataFrame, lay, col_name: str, clone_col="clone_id", chr_col="chr",
                          start_col="start", cn_state_col="state"):
    """consensus_clone_profiles of a per-cell-block table (``lay`` from _block_layout) from its
    blocks as they lie (``consensus_arrays``: the order of cells and loci does not matter), as
    the sorted copy's block path returns it -- index (chr as CHR_ORDER categories, start), sorted
    -- without the copy; None where the general path is needed."""
    B, L, bp, q, ch0 = lay
    fast = consensus_arrays(cn[clone_col].to_numpy(), cn[col_name].to_numpy(np.float64),
                            None if cn_state_col is None else cn[cn_state_col].to_numpy(), B, L)
    if fast is None:
        return None
    med, ku = fast
    chr_lab = pd.Categorical(np.array(CHR_ORDER, dtype=object)[ch0[q]], categories=CHR_ORDER)
    idx = pd.MultiIndex.from_arrays([chr_lab, cn[start_col].to_numpy()[:L][q]], names=[chr_col, start_col])
    prof = pd.DataFrame(med[q], index=idx, columns=pd.Index(ku, name=clone_col))
    return prof.dropna(how="all").dropna(axis=1, how="all").sort_index()


def consensus_clone_profiles(cn: pd.DataFrame, col_name: str, clone_col="clone_id", cell_col="cell_id",
                             chr_col="chr", start_col="start", cn_state_col="state", keys=None) -> pd.DataFrame:
    """compute_consensus_clone_profiles (:42-88): median of ``col_name`` per (locus, clone)
    over the clone's majority-ploidy cells; index (chr, start) sorted as pivot_table sorts
    it, columns the sorted clone ids.  Integer codes, row masks and one lexsort; the long
    table itself is never copied.  A DeferredTable is taken from its source's blocks
    (``consensus_from_blocks``) when they qualify, else from its sorted copy."""
    if isinstance(cn, DeferredTable):
        prof = consensus_from_blocks(cn.source, cn.lay, col_name, clone_col=clone_col, chr_col=chr_col,
                                     start_col=start_col, cn_state_col=cn_state_col)
        if prof is not None:
            return prof
        cn = cn.result()
    if (isinstance(keys, RegularKeys) and _n_rows(keys) == len(cn)
            and isinstance(cn[chr_col].dtype, pd.CategoricalDtype)):
        fast = _consensus_blocks(cn, col_name, clone_col, cn_state_col, keys)
        if fast is not None:
            med, ku = fast
            chr_lab = pd.Categorical(keys.loci_chr, categories=cn[chr_col].cat.categories,
                                     ordered=cn[chr_col].cat.ordered)
            idx = pd.MultiIndex.from_arrays([chr_lab, keys.loci_start], names=[chr_col, start_col])
            prof = pd.DataFrame(med, index=idx, columns=pd.Index(ku, name=clone_col))
            return prof.dropna(how="all").dropna(axis=1, how="all").sort_index()
    kc, ku = _sorted_codes(cn[clone_col].to_numpy())
    if "None" in set(ku.tolist()):                       # clone 'None' is removed (:63)
        bad = int(np.flatnonzero(ku == "None")[0])
        kc = np.where(kc == bad, -1, kc)
    rows = kc >= 0
    if cn_state_col is not None:
        if keys is not None and _n_rows(keys) == len(cn):
            cc, cells = keys.cell_code, keys.cells
        else:
            cc, cells = _sorted_codes(cn[cell_col].to_numpy())
        cc = np.where(rows, cc, -1)
        rows &= _majority_ploidy_rows(cn, clone_col, cell_col, cn_state_col, cc, len(cells), kc, len(ku))
    if keys is not None and _n_rows(keys) == len(cn) and isinstance(cn[chr_col].dtype, pd.CategoricalDtype):
        # the sorted table's locus codes (sorted (chr category, start) uniques), no re-hashing
        lc = keys.locus_code
        ok = lc >= 0
        n_loci = keys.loci_start.size
        chr_lab, start_lab = keys.loci_chr, keys.loci_start
        valid_l = np.ones(n_loci, bool)
    else:
        hc, hu = _factorize(cn[chr_col].to_numpy())
        st = cn[start_col].to_numpy()
        ok = hc >= 0
        lc, lu = pd.factorize(np.where(ok, hc.astype(np.int64) * (1 << 40) + np.where(ok, st, 0).astype(np.int64), -1))
        n_loci = len(lu)
        hu_arr = np.asarray(hu, dtype=object)
        chr_lab = hu_arr[(lu >> 40).astype(np.int64) % max(len(hu_arr), 1)]
        start_lab = lu & ((1 << 40) - 1)
        valid_l = np.asarray(lu) >= 0
    grp = np.where(rows & ok, lc * len(ku) + kc, -1)
    med = _group_median(grp, cn[col_name].to_numpy(np.float64), n_loci * len(ku))
    if isinstance(cn[chr_col].dtype, pd.CategoricalDtype):
        chr_lab = pd.Categorical(chr_lab, categories=cn[chr_col].cat.categories, ordered=cn[chr_col].cat.ordered)
    idx = pd.MultiIndex.from_arrays([chr_lab, start_lab], names=[chr_col, start_col])
    prof = pd.DataFrame(med.reshape(n_loci, len(ku)), index=idx, columns=pd.Index(ku, name=clone_col))
    prof = prof[valid_l].dropna(how="all").dropna(axis=1, how="all")
    return prof.sort_index()


def first_clone(cn: pd.DataFrame, cells, cell_col="cell_id", clone_col="clone_id", keys=None) -> np.ndarray:
    """cn.loc[cn[cell]==id][clone].values[0] for every id (pert_model.py:289-290).
    ``keys``: the table's TableKeys (row order), to find first rows by cell code."""
    if isinstance(cn, DeferredTable) and not (isinstance(keys, RegularKeys) and _n_rows(keys) == len(cn)):
        cn = cn.result()
    if keys is not None and _n_rows(keys) == len(cn):
        if isinstance(keys, RegularKeys):
            rows = np.arange(keys.cells.size) * keys.regular          # each cell's first row
        else:
            ok = keys.cell_code >= 0
            _, first = np.unique(keys.cell_code[ok], return_index=True)
            rows = np.flatnonzero(ok)[first]
        clone_of = (cn.column_at(clone_col, rows) if isinstance(cn, DeferredTable)
                    else cn[clone_col].to_numpy()[rows])              # per keys.cells
        pos = pd.Index(keys.cells).get_indexer(np.asarray(cells))
        out = np.empty(len(pos), dtype=object)
        out[pos >= 0] = clone_of[pos[pos >= 0]]
        out[pos < 0] = np.nan
        return out
    f = cn[[cell_col, clone_col]].drop_duplicates(cell_col).set_index(cell_col)[clone_col]
    return f.reindex(cells).to_numpy()


def _profile_columns(profiles: pd.DataFrame, clones, loci_chr, loci_start):
    """(the profiles at the fitted loci (L, n_profiles), each cell's profile column (N,))."""
    idx = pd.MultiIndex.from_arrays([profiles.index.get_level_values(0).astype(str),
                                     profiles.index.get_level_values(1)])
    li = idx.get_indexer(pd.MultiIndex.from_arrays([np.asarray(loci_chr).astype(str), loci_start]))
    if (li < 0).any():
        raise ValueError("clone profiles miss some loci of the fitted cells")
    cols = {c: j for j, c in enumerate(profiles.columns)}
    return profiles.to_numpy()[li], np.array([cols[c] for c in clones], dtype=np.int64)


def _profile_matrix(profiles: pd.DataFrame, clones, loci_chr, loci_start) -> np.ndarray:
    """(L, N): each cell's clone profile at the fitted loci (pert_model.py:289-293)."""
    mat, ci = _profile_columns(profiles, clones, loci_chr, loci_start)
    return np.take(mat, ci, axis=1)


# --------------------------------------------------------------------------- eta builders
def build_cn_prior(states, weight: float, P: int) -> EtaCodebook:
    """pert_model.py:272-282: ones, eta[l, n, state] = weight."""
    return EtaCodebook.from_states(np.asarray(states).astype(np.int64), weight, P)


def build_clone_cn_prior(cn: pd.DataFrame, cells, loci_chr, loci_start, profiles: pd.DataFrame, weight: float,
                         P: int, cell_col="cell_id", clone_col="clone_id", keys=None,
                         cell_range: slice = None) -> EtaCodebook:
    """pert_model.py:285-296: the consensus clone profile (int64-truncated) as prior state --
    truncated and range-checked per clone, then one uint16 gather of the clone columns
    (the same codes as build_cn_prior on the (L, N) profile matrix).  ``cell_range``: the
    code book of that contiguous range of ``cells`` only (a rank's shard)."""
    clones = first_clone(cn, cells, cell_col, clone_col, keys)
    mat, ci = _profile_columns(profiles, clones, loci_chr, loci_start)
    st = mat.astype(np.int64)
    used = st[:, np.unique(ci)]          # every cell's clone: each rank of a sharded fit raises alike
    if used.size and (used.min() < 0 or used.max() >= P):      # before the uint16 narrowing
        raise ValueError("CN states must lie in [0, P) for P={}".format(P))
    if cell_range is not None:
        ci = ci[cell_range]
    return EtaCodebook.from_states(np.take(st.astype(np.uint16), ci, axis=1), weight, P)


def pearson_columns(A: np.ndarray, B: np.ndarray) -> np.ndarray:
    """Pearson r between every column of A (L, n) and of B (L, m) (scipy.stats.pearsonr)."""
    import torch
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    a = torch.as_tensor(A, dtype=torch.float64, device=dev)
    b = torch.as_tensor(B, dtype=torch.float64, device=dev)
    a = a - a.mean(0, keepdim=True)
    b = b - b.mean(0, keepdim=True)
    a = a / a.norm(dim=0, keepdim=True)
    b = b / b.norm(dim=0, keepdim=True)
    return (a.T @ b).cpu().numpy()


def compute_cell_corrs(s_cell_cn: pd.DataFrame, clone_cn_g1: pd.DataFrame, s_cell_id, col='rpm_gc_norm',
                       cell_col='cell_id', chr_col='chr', start_col='start') -> pd.DataFrame:
    """compute_cell_corrs (normalize_by_cell.py:148-180) for one S cell: Pearson r and its
    p-value (scipy.stats.pearsonr) between ``col`` of the S cell and of every G1 cell of
    ``clone_cn_g1`` over the loci both have rows for, G1 cells in ``groupby`` (sorted id)
    order, then sorted by r descending with pandas' default sort (NaN r last).  The
    correlation-matched priors use the batched equivalent (``g1_cell_matches``)."""
    from scipy.stats import pearsonr
    s_key = pd.MultiIndex.from_arrays([s_cell_cn[chr_col].astype(str).to_numpy(), s_cell_cn[start_col].to_numpy()])
    s_val = pd.Series(s_cell_cn[col].to_numpy(np.float64), index=s_key)
    rows = []
    for g1_cell_id, grp in clone_cn_g1.groupby(cell_col):
        g_key = pd.MultiIndex.from_arrays([grp[chr_col].astype(str).to_numpy(), grp[start_col].to_numpy()])
        pos = s_key.get_indexer(g_key)
        hit = pos >= 0
        x = s_val.to_numpy()[pos[hit]]
        y = grp[col].to_numpy(np.float64)[hit]
        import warnings
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            r, p = pearsonr(x, y)
        rows.append((s_cell_id, g1_cell_id, float(r), float(p)))
    out = pd.DataFrame(rows, columns=['s_cell_id', 'g1_cell_id', 'pearson_r', 'pearson_pval'])
    return out.sort_values(by=['pearson_r'], ascending=False)


def rank_desc_like_pandas(vals: np.ndarray) -> np.ndarray:
    """Row-wise ``DataFrame.sort_values(ascending=False)`` order (default quicksort, NaNs
    last) as the reference ranks its correlation table (normalize_by_cell.py:177-178):
    pandas' ``nargsort`` reverses the non-NaN values, argsorts them with numpy's quicksort
    and reverses the result, so ties come out in the order that procedure gives, which is
    not the stable one.  NaN-free rows are done as one 2-D argsort; rows holding NaN go
    through pandas' nargsort itself."""
    from pandas.core.sorting import nargsort
    vals = np.asarray(vals, dtype=np.float64)
    n_rows, n = vals.shape
    out = np.empty((n_rows, n), dtype=np.int64)
    nan_rows = np.isnan(vals).any(axis=1)
    ok = ~nan_rows
    if ok.any():
        rev = vals[ok][:, ::-1]
        o = np.argsort(rev, axis=1, kind="quicksort")
        out[ok] = (n - 1 - o)[:, ::-1]
    for r in np.flatnonzero(nan_rows):
        out[r] = nargsort(vals[r], kind="quicksort", ascending=False, na_position="last")
    return out


def g1_cell_matches(inp: PertInputs, cn_s: pd.DataFrame, cn_g1: pd.DataFrame, J: int, cell_col="cell_id",
                    clone_col: Optional[str] = "clone_id", g1_pool: Optional[pd.DataFrame] = None):
    """For each S cell, its J best-matching G1 cells (pert_model.py:322-345, :677-695):
    the G1 cells of the S cell's clone in the pool (``cn_g1`` or the majority-ploidy
    ``g1_pool``), ranked by the Pearson r of ``input_col`` between the two cells
    (compute_cell_corrs, normalize_by_cell.py:148-180), best first.  Returns an (Ns, J)
    index array into ``inp.cells_g``.

    The reference correlates each pair over the loci the two cells' rows share (a merge
    on chr/start of the long tables); its prior assignment then writes the matched G1
    cell's state rows into the fitted (complete) loci positionally, which only succeeds
    when that cell's rows are exactly those loci -- so wherever the reference runs, the
    shared loci are the fitted loci and the pivot's correlations are its correlations.
    Candidates are ranked in ``groupby(cell_col)`` order (sorted cell ids, the pivot's
    order) with pandas' sort (``rank_desc_like_pandas``), ties and NaN r included.
    Raises as the reference does when an S cell's clone has no G1 cell in the pool
    (ValueError, ``pd.concat`` of nothing) or fewer than J (IndexError, ``iloc[j]``)."""
    pool = cn_g1 if g1_pool is None else g1_pool
    allowed = pd.Index(inp.cells_g).isin(pool[cell_col].unique())
    rs = inp.reads_s if inp.reads_s_raw is None else inp.reads_s_raw
    rg = inp.reads_g if inp.reads_g_raw is None else inp.reads_g_raw
    corr = pearson_columns(np.asarray(rs, np.float64), np.asarray(rg, np.float64))
    if clone_col is not None:
        cs = pd.Series(first_clone(cn_s, inp.cells_s, cell_col, clone_col))
        cg = pd.Series(first_clone(pool, inp.cells_g, cell_col, clone_col))
        gkey, guniq = pd.factorize(cg)                              # NaN clone -> -1
        skey = pd.Index(guniq).get_indexer(cs)                      # S clones unknown to G1 -> -1
        groups = [(np.flatnonzero(skey == k), np.flatnonzero((gkey == k) & allowed)) for k in range(len(guniq))]
        missing = np.flatnonzero(skey < 0)
    else:
        groups = [(np.arange(corr.shape[0]), np.flatnonzero(allowed))]
        missing = np.array([], dtype=np.int64)
    for k, (srows, gcols) in enumerate(groups):
        if srows.size and gcols.size == 0:
            missing = np.concatenate([missing, srows])
    if missing.size:
        raise ValueError("No objects to concatenate: S cell {} has no G1 cell of its clone to correlate with "
                         "(compute_cell_corrs)".format(inp.cells_s[int(missing[0])]))
    out = np.empty((corr.shape[0], J), dtype=np.int64)
    for srows, gcols in groups:
        if srows.size == 0:
            continue
        if gcols.size < J:
            raise IndexError("single positional indexer is out-of-bounds: the clone of S cell {} has {} G1 "
                             "cells in the pool, fewer than J = {}".format(inp.cells_s[int(srows[0])],
                                                                          gcols.size, J))
        order = rank_desc_like_pandas(corr[np.ix_(srows, gcols)])[:, :J]
        out[srows] = gcols[order]
    return out


def build_g1_cells_prior(inp: PertInputs, cn_s, cn_g1, weight: float, P: int, cell_col="cell_id",
                         clone_col="clone_id") -> EtaCodebook:
    """The ``g1_cells`` branch (pert_model.py:671-701): the best-correlated G1 cell of the
    S cell's clone (every G1 cell, no ploidy filter) gives the prior state profile."""
    best = g1_cell_matches(inp, cn_s, cn_g1, 1, cell_col, clone_col)[:, 0]
    return build_cn_prior(inp.states_g[:, best].astype(np.int64), weight, P)


def _composite_pool(cn_g1: pd.DataFrame, clone_col: str, cell_col: str, cn_state_col: str,
                    ploidy_col: str = "ploidy") -> pd.DataFrame:
    """The G1 rows build_composite_cn_prior draws matches from (pert_model.py:312-317):
    add_cell_ploidies unless the table already has a ``ploidy`` column, then filter_ploidies
    (the majority ploidy of each clone, ties to the smallest; rows of a NaN clone dropped)."""
    if ploidy_col in cn_g1.columns:
        return filter_ploidies(cn_g1, clone_col=clone_col, cell_col=cell_col, cn_state_col=cn_state_col,
                               ploidy_col=ploidy_col)
    return cn_g1[_majority_ploidy_rows(cn_g1, clone_col, cell_col, cn_state_col)]


def build_composite_cn_prior(inp: PertInputs, cn_s, cn_g1, profiles: pd.DataFrame, P: int, J: int = 5,
                             weight: float = 1e5, cell_col="cell_id", clone_col="clone_id",
                             cn_state_col="state") -> EtaCodebook:
    """build_composite_cn_prior (pert_model.py:299-361): ones + weight*J*2 at the clone
    consensus state + weight*(J-j) at the j-th best-matching G1 cell's state (G1 cells of
    the majority ploidy of the clone; J capped by the smallest clone, counted before the
    ploidy filter as the reference counts it)."""
    if clone_col is not None:
        sizes = cn_g1[[cell_col, clone_col]].drop_duplicates().groupby(clone_col).size()
        J = int(min(J, sizes.min()))
        pool = _composite_pool(cn_g1, clone_col, cell_col, cn_state_col)
    else:
        pool = cn_g1
    match = g1_cell_matches(inp, cn_s, cn_g1, J, cell_col, clone_col, g1_pool=pool)     # (Ns, J)
    clones = first_clone(cn_s, inp.cells_s, cell_col, clone_col)
    clone_state = _profile_matrix(profiles, clones, inp.loci_chr, inp.loci_start).astype(np.int64)
    g_states = inp.states_g.astype(np.int64)
    L, Ns = clone_state.shape
    keys = clone_state.copy()
    cols = [clone_state]
    for j in range(J):
        sj = g_states[:, match[:, j]]
        cols.append(sj)
        keys = keys * P + sj
    if (np.stack(cols).max() >= P) or (np.stack(cols).min() < 0):
        raise ValueError("CN states must lie in [0, P)")
    ukeys, inv = np.unique(keys.reshape(-1), return_inverse=True)
    if ukeys.size > 65535:
        raise ValueError("composite prior has more than 65535 distinct rows")
    first = np.zeros(ukeys.size, dtype=np.int64)
    first[inv[::-1]] = np.arange(inv.size)[::-1]
    flat = [c.reshape(-1)[first] for c in cols]
    table = np.ones((ukeys.size, P), dtype=np.float32)
    rows = np.arange(ukeys.size)
    table[rows, flat[0]] += np.float32(weight * J * 2)
    for j in range(J):
        table[rows, flat[1 + j]] += np.float32(weight * (J - j))
    return EtaCodebook(inv.reshape(L, Ns).astype(np.uint16), table)


def diploid_prior(L: int, N: int, weight: float, P: int) -> EtaCodebook:
    return build_cn_prior(np.full((L, N), 2, dtype=np.int64), weight, P)


def uniform_prior(L: int, N: int, P: int) -> EtaCodebook:
    """pert_model.py:716: eta = 1/P everywhere (ploidy then averages argmax = 0)."""
    return EtaCodebook(np.zeros((L, N), np.uint16), np.full((1, P), np.float32(1.0) / np.float32(P), np.float32))


# --------------------------------------------------------------------------- tau init
def manhattan_binarization(X: np.ndarray, MEAN_GAP_THRESH=0.7, EARLY_S_SKEW_THRESH=0.2,
                           LATE_S_SKEW_THRESH=-0.2):
    """pert_model.py:364-423 (one cell), threshold scan vectorised."""
    from scipy.stats import skew
    from sklearn.mixture import GaussianMixture
    X = (X - np.mean(X)) / np.std(X)
    gm = GaussianMixture(n_components=2, random_state=0)
    gm.fit_predict(X)
    mean_0, mean_1 = gm.means_[0][0], gm.means_[1][0]
    mean_gap = abs(mean_0 - mean_1)
    b0, b1 = min(mean_0, mean_1), max(mean_0, mean_1)
    X = X.flatten()
    if mean_gap < MEAN_GAP_THRESH:
        cell_skew = skew(X)
        if cell_skew > EARLY_S_SKEW_THRESH:
            b0, b1 = np.percentile(X, 50), np.percentile(X, 95)
        elif cell_skew < LATE_S_SKEW_THRESH:
            b0, b1 = np.percentile(X, 5), np.percentile(X, 50)
        else:
            b0, b1 = np.percentile(X, 25), np.percentile(X, 75)
    threshs = np.linspace(b0, b1, 100)
    B = np.where(X[None, :] > threshs[:, None], b1, b0)
    dists = np.abs(X[None, :] - B).sum(axis=1)
    best_t = threshs[int(np.argmin(dists))]           # first minimum, like the strict '<' scan
    cell_rt = np.where(X > best_t, 1, 0)
    return cell_rt, cell_rt.sum() / len(cell_rt)


def guess_times(reads: np.ndarray, cn_states: np.ndarray, upsilon: float = 6, n_jobs: int = 1):
    """pert_model.py:426-457: t_init, t_alpha_prior, t_beta_prior per cell.

    The cells are fitted one after another, as the reference loops over them, whatever
    ``n_jobs`` says (kept for the signature): GaussianMixture's k-means runs inside
    sklearn's per-call threadpoolctl limit, and that limit, entered from several threads of
    one process at once, races OpenBLAS's thread-count setter against the other threads'
    BLAS calls (a 10k-cell run deadlocked on it)."""
    import torch
    del n_jobs
    x = torch.as_tensor(reads, dtype=torch.float32)
    st = torch.as_tensor(cn_states, dtype=torch.float32)
    half = (torch.ones(x.shape) * 0.5).type(torch.float32)
    norm = (x / torch.where(st > 0.0, st, half)).numpy()
    fr = [manhattan_binarization(norm[:, i].reshape(-1, 1)) for i in range(norm.shape[1])]
    t_init = np.array([f[1] for f in fr], dtype=np.float32)
    alpha = (t_init * upsilon).astype(np.float32)
    return t_init, alpha, (upsilon - alpha).astype(np.float32)


def make_g1_g2_training_data(states_g, reads_g, libs_g):
    """pert_model.py:228-251: every G1/2 cell twice, rep = 0 then rep = 1."""
    states = np.concatenate([states_g, states_g], axis=1)
    reads = np.concatenate([reads_g, reads_g], axis=1)
    libs = np.concatenate([libs_g, libs_g])
    rep = np.concatenate([np.zeros(states_g.shape), np.ones(states_g.shape)], axis=1)
    return states, reads, libs, rep
