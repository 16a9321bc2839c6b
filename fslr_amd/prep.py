"""Host-side preparation of the hot path's input (vectorised numpy / pandas).

Everything here runs once per input on the host, in front of the device path:

* ``fillings_mask`` / ``qlen2``   — keep_fillings (cluster.py:14-31)
* ``data_order``                  — prepare_data's ``sort_values('start')``
                                    (cluster.py:114; pandas' default quicksort
                                    argsort of the int64 column, ties included)
* ``mask_keep``                   — mask_sequences2 (cluster.py:89-106)
* ``IntervalData``                — the prepared ``data`` list as columns; it still
                                    behaves as a sequence of ``IntervalItem``
* ``build_csr``                   — ranks and per-read lists (cluster.py:189-191)
* ``fold_overlap_threshold``      — integer form of ``calculate_overlap >= overlap``
                                    (cluster.py:133-136, 157)
* ``pass_table``                  — Jaccard cut lookup (cluster.py:216-219)

The integer folds are exact: Python float division of two ints below 2**53 is
the correctly rounded IEEE quotient, numpy float64 division is the same
operation, and ``fl(o/a)`` is monotone in ``o``, so ``fl(o/a) >= p`` holds on an
integer interval of ``o`` whose end points are found by searching around
``p*a`` with the very same division.
"""
from __future__ import annotations

import dataclasses
import math
from collections import namedtuple

import numpy as np

from ._lib import FSLR_MAX_L, FSLR_MAX_READS, FSLR_THR_ZERO_ALN, PASS_STRIDE

IntervalItem = namedtuple('interval_item',
                          ['chrom', 'start', 'end', 'aln_size', 'qname', 'n_alignments', 'qlen2', 'middle', 'index'])

THR_NEVER = np.iinfo(np.int32).max
MAX_COORD = 1 << 30


# ------------------------------------------------------------------------------------------
# keep_fillings (cluster.py:14-31)
# ------------------------------------------------------------------------------------------
def first_last_masks(codes: np.ndarray):
    """Row masks of the first and the last row of every group code (file order)."""
    n = codes.shape[0]
    first = np.zeros(n, dtype=bool)
    last = np.zeros(n, dtype=bool)
    if n == 0:
        return first, last
    codes = np.asarray(codes)
    # fast path, O(n): every code's rows form one contiguous run (a BED sorted by qname, as
    # collect_mapping_info.py:174 writes it) -> first / last rows are the run boundaries
    brk = np.flatnonzero(codes[1:] != codes[:-1]) + 1
    starts = np.concatenate(([0], brk))
    if codes.dtype.kind in 'iu' and codes.min() >= 0 and codes.max() < 4 * n + 1024:
        n_distinct = int(np.count_nonzero(np.bincount(codes)))
    else:
        n_distinct = int(np.unique(codes[starts]).size) if starts.size < n else n
    if n_distinct == starts.size:
        first[starts] = True
        last[np.concatenate((brk - 1, [n - 1]))] = True
        return first, last
    _, fi = np.unique(codes, return_index=True)
    _, li = np.unique(codes[::-1], return_index=True)
    first[fi] = True
    last[n - 1 - li] = True
    return first, last


def group_span(codes: np.ndarray, qstart: np.ndarray, qend: np.ndarray, n_codes: int) -> np.ndarray:
    """max(qend) - min(qstart) per code (codes with no rows get 0)."""
    import pandas as pd
    s = pd.DataFrame({'c': codes, 'qs': qstart, 'qe': qend}).groupby('c', sort=False)
    mx = s['qe'].max()
    mn = s['qs'].min()
    out = np.zeros(n_codes, dtype=np.int64)
    out[mx.index.to_numpy()] = (mx - mn).to_numpy()
    return out


# ------------------------------------------------------------------------------------------
# prepared data (cluster.py:109-121)
# ------------------------------------------------------------------------------------------
@dataclasses.dataclass
class IntervalData:
    """The reference's ``data`` list (cluster.py:116-121) as columns, in list order.

    Iterating yields ``IntervalItem`` tuples like the reference; the device path
    only reads the numeric columns.
    """
    chrom: np.ndarray        # int64 numeric chromosome (rename_chromosomes ids)
    start: np.ndarray        # int64
    end: np.ndarray          # int64
    aln_size: np.ndarray     # int64
    qcode: np.ndarray        # int64 code into qnames
    qnames: np.ndarray       # object array: code → qname
    n_alignments: np.ndarray
    qlen2: np.ndarray
    middle: np.ndarray
    index: np.ndarray        # bed row labels
    _csr: object = None

    def __len__(self):
        return int(self.start.shape[0])

    def __getitem__(self, k):
        if isinstance(k, slice):
            return [self[i] for i in range(*k.indices(len(self)))]
        k = int(k)
        return IntervalItem(int(self.chrom[k]), int(self.start[k]), int(self.end[k]), int(self.aln_size[k]),
                            self.qnames[self.qcode[k]], int(self.n_alignments[k]), int(self.qlen2[k]),
                            int(self.middle[k]), self.index[k].item() if hasattr(self.index[k], 'item')
                            else self.index[k])

    def __iter__(self):
        for k in range(len(self)):
            yield self[k]

    def select(self, keep: np.ndarray) -> 'IntervalData':
        f = {f.name: getattr(self, f.name)[keep] for f in dataclasses.fields(self)
             if f.name not in ('qnames', '_csr')}
        return IntervalData(qnames=self.qnames, **f)

    def csr(self):
        if self._csr is None:
            self._csr = build_csr(self)
        return self._csr

    @classmethod
    def from_items(cls, items) -> 'IntervalData':
        """The columns of a reference-built ``data`` list (a sequence of ``IntervalItem``, the
        return value of the reference's prepare_data, cluster.py:116-121), in list order."""
        import pandas as pd
        items = list(items)
        n = len(items)
        cols = list(zip(*items)) if n else [()] * 9
        chrom_raw = np.asarray(cols[0], dtype=object) if n else np.zeros(0, object)
        try:
            chrom = np.asarray(cols[0], dtype=np.int64) if n else np.zeros(0, np.int64)
        except (TypeError, ValueError):                  # names (rename_chromosomes not applied)
            chrom = pd.factorize(chrom_raw, sort=False)[0].astype(np.int64)
        codes, uniq = pd.factorize(np.asarray(cols[4], dtype=object) if n else np.zeros(0, object), sort=False)
        i64 = lambda k: np.asarray(cols[k], dtype=np.int64) if n else np.zeros(0, np.int64)
        return cls(chrom=chrom, start=i64(1), end=i64(2), aln_size=i64(3), qcode=codes.astype(np.int64),
                   qnames=np.asarray(uniq, dtype=object), n_alignments=i64(5), qlen2=i64(6), middle=i64(7),
                   index=np.asarray(cols[8], dtype=object) if n else np.zeros(0, object))


def data_order(start: np.ndarray) -> np.ndarray:
    """Row order of ``df.sort_values('start')`` (pandas nargsort: quicksort argsort, no NaN).  When
    no two starts tie every sort gives that order, and a threaded radix sort makes it
    (ingest.argsort_distinct); ties keep numpy's quicksort, whose tie order pandas' is."""
    start = np.asarray(start, dtype=np.int64)
    if start.size >= 1 << 16:
        from . import ingest
        order = ingest.argsort_distinct(start)
        if order is not None:
            return order
    return start.argsort(kind='quicksort')


def mask_keep(chrom, start, end, mask, chromosome_lengths, threshold=500_000) -> np.ndarray:
    """Boolean keep mask of mask_sequences2 (cluster.py:89-106), vectorised."""
    n = chrom.shape[0]
    keep = np.ones(n, dtype=bool)
    if not mask:
        return keep
    ids = [m for m in mask if m != 'subtelomere' and m is not None and not isinstance(m, str)]
    if ids:
        keep &= ~np.isin(chrom, np.asarray(ids, dtype=np.int64))
    if 'subtelomere' in mask:
        long_ = {k: v for k, v in chromosome_lengths.items() if k is not None and v > 1_000_000}
        if long_ and n:
            cmax = int(max(max(long_), chrom.max(initial=0))) + 1
            lut = np.full(cmax + 1, -1, dtype=np.int64)
            for k, v in long_.items():
                if isinstance(k, (int, np.integer)) and 0 <= int(k) <= cmax:
                    lut[int(k)] = v
            c = np.clip(chrom, 0, cmax)
            L = np.where((chrom >= 0) & (chrom <= cmax), lut[c], -1)
            has = L >= 0
            keep &= ~(has & ((start < threshold) | (L - end < threshold)))
    return keep


# ------------------------------------------------------------------------------------------
# CSR (cluster.py:189-191)
# ------------------------------------------------------------------------------------------
@dataclasses.dataclass
class CSR:
    read_off: np.ndarray     # int32 [n+1]
    read_qlen2: np.ndarray   # int32 [n]
    read_nal: np.ndarray     # int32 [n]
    iv_chrom: np.ndarray     # int32 [ni] dense ids 0..n_chroms-1
    iv_start: np.ndarray     # int32
    iv_end: np.ndarray       # int32
    iv_aln: np.ndarray       # int64 aln_size (for threshold folds)
    n_chroms: int
    read_qcode: np.ndarray   # int64 [n] code of each rank's qname
    data_pos: np.ndarray     # int64 [ni] position in the data list
    nal_varies: bool         # n_alignments not constant within some read (order-dependent in the reference)
    start_sorted: bool = True  # the data list is in non-decreasing start order (prepare_data's sort)

    @property
    def n_reads(self):
        return int(self.read_off.shape[0] - 1)

    @property
    def n_intervals(self):
        return int(self.iv_start.shape[0])


def build_csr(data: IntervalData) -> CSR:
    n_iv = len(data)
    codes = np.asarray(data.qcode, dtype=np.int64)
    from . import ingest
    grouped = ingest.group_by_first_appearance(codes) if n_iv else None
    if grouped is not None:
        # one native O(n) pass: ranks by first appearance, counting-sort grouping
        read_qcode, off_g, perm = grouped
        counts = np.diff(off_g)
    elif n_iv:
        # rank = order of first appearance (cluster.py:189-191); codes are non-negative ints
        if codes.min() >= 0 and codes.max() < 4 * n_iv + 1024:
            first_at = np.full(int(codes.max()) + 1, n_iv, dtype=np.int64)
            np.minimum.at(first_at, codes, np.arange(n_iv, dtype=np.int64))
            uniq = np.flatnonzero(first_at < n_iv)
            first = first_at[uniq]
        else:
            uniq, first = np.unique(codes, return_index=True)
        order = np.argsort(first, kind='stable')
        rank_of = np.empty(int(uniq.max()) + 1, dtype=np.int64)
        rank_of[uniq[order]] = np.arange(uniq.size, dtype=np.int64)
        rank = rank_of[codes]
        # stable grouping by rank == sort of the distinct keys rank << 32 | data position
        key = (rank << 32) | np.arange(n_iv, dtype=np.int64)
        key.sort()
        perm = key & 0xFFFFFFFF
        del key
        counts = np.bincount(rank, minlength=uniq.size)
        read_qcode = uniq[order]
    else:
        rank = perm = np.zeros(0, dtype=np.int64)
        counts = np.zeros(0, dtype=np.int64)
        read_qcode = np.zeros(0, dtype=np.int64)
    n = counts.size
    if n >= FSLR_MAX_READS:
        raise ValueError(f'{n} reads exceed the device limit of {FSLR_MAX_READS}')
    # reads of more than FSLR_MAX_L intervals are uploaded split into chunks (fslr_set_reads_any;
    # split_long_reads below is the same layout on the host)
    off = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(counts, out=off[1:])
    start, end, chrom_raw, aln_p, nal_p = ingest.gather_columns(
        [data.start, data.end, data.chrom, data.aln_size, data.n_alignments], perm) if n_iv else \
        [np.zeros(0, np.int64)] * 5
    if n_iv and (start.min() < 0 or end.max() >= MAX_COORD):
        raise ValueError('interval coordinates must lie in [0, 2**30) for the device path')
    if n_iv and chrom_raw.min() >= 0 and chrom_raw.max() < (1 << 24):
        present = np.bincount(chrom_raw) > 0          # chromosome ids are small ints: O(n) dense ids
        cids = np.flatnonzero(present)
        chrom_dense = (np.cumsum(present) - 1)[chrom_raw]
    elif n_iv:
        cids, chrom_dense = np.unique(chrom_raw, return_inverse=True)
    else:
        cids, chrom_dense = np.zeros(0), np.zeros(0, np.int64)
    first_iv = perm[off[:-1]] if n else np.zeros(0, dtype=np.int64)
    qlen2 = np.asarray(data.qlen2, np.int64)
    nal = np.asarray(data.n_alignments, np.int64)
    read_qlen2 = qlen2[first_iv]
    read_nal = nal[first_iv]
    for name, v in (('qlen2', read_qlen2), ('n_alignments', read_nal)):
        if v.size and (v.min() < np.iinfo(np.int32).min or v.max() > np.iinfo(np.int32).max):
            raise ValueError(f'{name} outside int32')
    nal_varies = bool(n_iv and np.any(nal_p != np.repeat(read_nal, counts)))
    return CSR(read_off=off.astype(np.int32), read_qlen2=read_qlen2.astype(np.int32),
               read_nal=read_nal.astype(np.int32), iv_chrom=chrom_dense.astype(np.int32),
               iv_start=start.astype(np.int32), iv_end=end.astype(np.int32),
               iv_aln=aln_p, n_chroms=max(1, int(len(cids))),
               read_qcode=read_qcode, data_pos=perm.astype(np.int64), nal_varies=nal_varies,
               start_sorted=bool(n_iv < 2 or np.all(np.diff(np.asarray(data.start, np.int64)) >= 0)))


def has_long_reads(csr: CSR) -> bool:
    return bool(csr.n_reads and np.diff(csr.read_off).max() > FSLR_MAX_L)


def split_long_reads(csr: CSR):
    """The virtual CSR of fslr_set_long_reads (include/fslr_hip.h): virtual read r < n
    is real read r with its first FSLR_MAX_L intervals; the further FSLR_MAX_L-interval chunks of the
    long reads follow as reads n, n+1, ... (in real-rank, then chunk order).  Returns
    (virtual CSR, vreal, vbase, rlen)."""
    L = np.diff(csr.read_off.astype(np.int64))
    n, ni = L.size, int(csr.read_off[-1])
    extra = np.maximum((L + FSLR_MAX_L - 1) // FSLR_MAX_L - 1, 0)
    n_extra = int(extra.sum())
    extra_off = np.zeros(n, np.int64)
    np.cumsum(extra[:-1], out=extra_off[1:])
    r_of = np.repeat(np.arange(n, dtype=np.int64), L)
    t = np.arange(ni, dtype=np.int64) - np.repeat(csr.read_off[:-1].astype(np.int64), L)
    chunk = t // FSLR_MAX_L
    v = np.where(chunk == 0, r_of, n + extra_off[r_of] + chunk - 1)
    perm = np.argsort(v, kind='stable')
    nv = n + n_extra
    voff = np.zeros(nv + 1, np.int64)
    np.cumsum(np.bincount(v, minlength=nv), out=voff[1:])
    xr = np.repeat(np.arange(n, dtype=np.int64), extra)
    vreal = np.concatenate([np.arange(n, dtype=np.int64), xr])
    xk = np.arange(n_extra, dtype=np.int64) - np.repeat(extra_off, extra) + 1
    vbase = np.concatenate([np.zeros(n, np.int64), xk * FSLR_MAX_L])
    vcsr = dataclasses.replace(
        csr, read_off=voff.astype(np.int32), read_qlen2=csr.read_qlen2[vreal], read_nal=csr.read_nal[vreal],
        iv_chrom=csr.iv_chrom[perm], iv_start=csr.iv_start[perm], iv_end=csr.iv_end[perm], iv_aln=csr.iv_aln[perm],
        read_qcode=csr.read_qcode[vreal], data_pos=csr.data_pos[perm])
    return vcsr, vreal.astype(np.int32), vbase.astype(np.int32), L.astype(np.int32)


def umax_table(cutoffs, max_i: int) -> np.ndarray:
    """``umax[I-1]`` = the largest U (I <= U <= 2 max_i) with ``I/U >= cutoff(I)`` in Python floats
    (cluster.py:216-219), or I - 1 when none passes: pass_table's rule for any I."""
    cut = list(cutoffs)
    if not cut:
        raise ValueError('min() arg is an empty sequence')
    hi = 2 * int(max_i)
    out = np.zeros(int(max_i), np.int64)
    for I in range(1, int(max_i) + 1):
        target = cut[I - 1] if I - 1 < len(cut) else cut[-1]
        if not I / I >= target:
            out[I - 1] = I - 1
            continue
        if I / hi >= target:
            out[I - 1] = hi
            continue
        u = max(I, min(hi, int(I / target)))       # I/U is decreasing in U: step to the boundary exactly
        while u > I and not I / u >= target:
            u -= 1
        while u < hi and I / (u + 1) >= target:
            u += 1
        out[I - 1] = u
    return out.astype(np.int32)


# ------------------------------------------------------------------------------------------
# exact integer folds of the float predicates
# ------------------------------------------------------------------------------------------
def fold_overlap_threshold(aln, overlap) -> np.ndarray:
    """Per-interval integer threshold for ``o / aln >= overlap`` (o >= 0 integer).

    Encoding (include/fslr_hip.h): ``t >= 0``: accept iff ``o >= t``; ``t < 0``:
    accept iff ``o <= ~t``; ``FSLR_THR_ZERO_ALN`` for ``aln == 0`` (the reference
    raises ZeroDivisionError when it evaluates such an interval).
    """
    a = np.asarray(aln, dtype=np.int64)
    p = float(overlap)
    if a.size > (1 << 16):
        lo, hi = int(a.min()), int(a.max())
        if lo >= 0 and hi < (1 << 22) and hi < a.size:
            # the fold is a function of the value: fold each value 0 .. max once, then one gather
            return fold_overlap_threshold(np.arange(hi + 1, dtype=np.int64), p)[a]
    out = np.full(a.shape, THR_NEVER, dtype=np.int64)
    out[a == 0] = FSLR_THR_ZERO_ALN
    pos = a > 0
    neg = a < 0
    if math.isnan(p):
        return out.astype(np.int32)
    if pos.any():
        ap = a[pos].astype(np.float64)
        if p <= 0.0:
            out[pos] = 0
        else:
            t = np.ceil(np.minimum(p * ap, 2.0 ** 40)).astype(np.int64)
            live = t <= MAX_COORD + 2          # beyond: no overlap of coordinates < 2**30 can reach it
            tl, al = t[live], ap[live]
            for _ in range(64):
                dec = (tl > 0) & ((tl - 1) / al >= p)
                inc = ~((tl / al) >= p)
                if not dec.any() and not inc.any():
                    break
                tl = tl - dec + inc
            else:  # pragma: no cover
                raise RuntimeError('threshold fold did not converge')
            t[live] = tl
            t = np.where(t >= MAX_COORD, THR_NEVER, t)
            out[pos] = t
    if neg.any() and p <= 0.0:
        an = (-a[neg]).astype(np.float64)
        q = -p
        h = np.floor(np.minimum(q * an, 2.0 ** 40)).astype(np.int64)
        live = h < MAX_COORD                   # beyond: every overlap below 2**30 is accepted
        hl, al = h[live], an[live]
        for _ in range(64):
            inc = (hl + 1) / al <= q
            dec = (hl > 0) & ~(hl / al <= q)
            if not inc.any() and not dec.any():
                break
            hl = hl + inc - dec
        else:  # pragma: no cover
            raise RuntimeError('threshold fold did not converge')
        h[live] = hl
        h = np.minimum(h, MAX_COORD)
        out[neg] = ~h
    return out.astype(np.int32)


def pass_table(cutoffs) -> np.ndarray:
    """``pass[I-1][U-1] = (I/U >= cutoff(I))`` with Python floats (cluster.py:216-219)."""
    cut = list(cutoffs)
    if not cut:
        raise ValueError('min() arg is an empty sequence')
    tab = np.zeros((FSLR_MAX_L, PASS_STRIDE), dtype=np.uint8)
    for I in range(1, FSLR_MAX_L + 1):
        target = cut[I - 1] if I - 1 < len(cut) else cut[-1]
        for U in range(I, PASS_STRIDE + 1):
            tab[I - 1, U - 1] = 1 if I / U >= target else 0
    return tab.reshape(-1)
