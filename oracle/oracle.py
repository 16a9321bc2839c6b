"""Python side of the CPU oracle (TEST INFRASTRUCTURE ONLY).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg import this module, and only as the checker.  The product package
``fslr_amd`` never imports it.

* ``restate_prep``   — restates the host stages in front of the hot loop with
  plain Python loops (small inputs only): ``main.py:211-216`` (mask option),
  ``cluster.py:14-31`` keep_fillings, ``cluster.py:109-121`` prepare_data,
  ``cluster.py:89-106`` mask_sequences2, ``cluster.py:189-191`` read ranks.
* ``run_core``       — ctypes call of ``fslr_oracle.c:oracle_query``
  (``cluster.py:187-234``).
* ``restate_numbering`` — ``main.py:247-342``: component index → cluster id,
  singletons numbered after in first-appearance order, float columns when any
  singleton exists.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, 'liboracle.so')

ORACLE_OK, ORACLE_ZERO_DIVISION, ORACLE_EDGE_CAPACITY, ORACLE_NOMEM, ORACLE_BAD_INPUT = range(5)


class _Input(ctypes.Structure):
    _fields_ = [('n_reads', ctypes.c_int64)] + [
        (f, ctypes.c_void_p) for f in ('read_off', 'chrom', 'start', 'end', 'aln', 'qlen2', 'nal', 'data_pos')]


class _Params(ctypes.Structure):
    _fields_ = [('overlap', ctypes.c_double), ('cutoffs', ctypes.c_void_p), ('n_cutoffs', ctypes.c_int64),
                ('qlen_diff', ctypes.c_double), ('nal_diff', ctypes.c_double),
                ('edge_threshold', ctypes.c_int64), ('use_cap', ctypes.c_int64), ('query_end', ctypes.c_int64)]


class _Stats(ctypes.Structure):
    _fields_ = [(f, ctypes.c_int64) for f in ('evaluated_pairs', 'jaccard_evals', 'interval_hits', 'n_edges',
                                              'max_fwd', 'n_components', 'err_a', 'err_b')]


_lib = None


def build() -> str:
    subprocess.run(['make', '-s', '-C', HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        for fn in (L.oracle_query, L.oracle_query_lean):
            fn.restype = ctypes.c_int
            fn.argtypes = [ctypes.POINTER(_Input), ctypes.POINTER(_Params)] + [ctypes.c_void_p] * 4 + [
                ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(_Stats)]
        L.oracle_jaccard_lists.restype = ctypes.c_int
        L.oracle_jaccard_lists.argtypes = [ctypes.c_int64] + [ctypes.c_void_p] * 4 + [ctypes.c_int64] + \
            [ctypes.c_void_p] * 4 + [ctypes.c_double, ctypes.c_void_p, ctypes.c_void_p]
        L.oracle_count_threads.restype = ctypes.c_int
        L.oracle_count_threads.argtypes = [ctypes.POINTER(_Input), ctypes.POINTER(_Params), ctypes.c_int64,
                                           ctypes.c_int64, ctypes.POINTER(_Stats)]
        L.oracle_lengths_differ.restype = ctypes.c_int
        L.oracle_lengths_differ.argtypes = [ctypes.c_int64] * 4 + [ctypes.c_double] * 2 + [ctypes.c_void_p]
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


class OracleCSR:
    """Rank-ordered CSR of the prepared intervals (what cluster.py:189-191 builds)."""

    def __init__(self, read_off, chrom, start, end, aln, qlen2, nal, data_pos, qnames=None):
        self.read_off = np.ascontiguousarray(read_off, dtype=np.int64)
        self.chrom = np.ascontiguousarray(chrom, dtype=np.int64)
        self.start = np.ascontiguousarray(start, dtype=np.int64)
        self.end = np.ascontiguousarray(end, dtype=np.int64)
        self.aln = np.ascontiguousarray(aln, dtype=np.int64)
        self.qlen2 = np.ascontiguousarray(qlen2, dtype=np.int64)
        self.nal = np.ascontiguousarray(nal, dtype=np.int64)
        self.data_pos = np.ascontiguousarray(data_pos, dtype=np.int64)
        self.qnames = qnames

    @property
    def n_reads(self):
        return int(self.read_off.shape[0] - 1)


class OracleZeroDivision(ZeroDivisionError):
    pass


def run_core(csr: OracleCSR, overlap=0.8, cutoffs=(1, 1, 0.66, 0.66, 0.66, 0.5), qlen_diff=0.04,
             n_aln_diff=0.25, edge_threshold=10, use_cap=True, query_end=-1, lean=False):
    """Run ``oracle_query``; returns dict with edges, fwd counts, component per read, stats.

    ``lean`` runs ``oracle_query_lean`` (the same seen-set held per read: full-size inputs).

    ``query_end`` >= 0 restricts the driver to query reads [0, query_end) (a bounded
    sample for the CPU baseline; components are then those of the sampled edges).
    """
    L = lib()
    N = csr.n_reads
    inp = _Input(N, *(_p(getattr(csr, f)) for f in ('read_off', 'chrom', 'start', 'end', 'aln', 'qlen2', 'nal',
                                                     'data_pos')))
    cut = np.ascontiguousarray(cutoffs, dtype=np.float64)
    prm = _Params(float(overlap), _p(cut), len(cut), float(qlen_diff), float(n_aln_diff), int(edge_threshold),
                  1 if use_cap else 0, int(query_end))
    cap = max(1024, 16 * N)
    while True:
        ea = np.empty(cap, np.int64)
        eb = np.empty(cap, np.int64)
        eI = np.empty(cap, np.int32)
        eU = np.empty(cap, np.int32)
        fwd = np.zeros(max(N, 1), np.int32)
        comp = np.full(max(N, 1), -1, np.int32)
        st = _Stats()
        rc = (L.oracle_query_lean if lean else L.oracle_query)(ctypes.byref(inp), ctypes.byref(prm), _p(ea), _p(eb), _p(eI), _p(eU), cap, _p(fwd),
                            _p(comp), ctypes.byref(st))
        if rc == ORACLE_EDGE_CAPACITY:
            cap *= 4
            continue
        break
    if rc == ORACLE_ZERO_DIVISION:
        raise OracleZeroDivision('division by zero')
    if rc != ORACLE_OK:
        raise RuntimeError(f'oracle_query failed rc={rc}')
    ne = st.n_edges
    return dict(edge_a=ea[:ne].copy(), edge_b=eb[:ne].copy(), edge_I=eI[:ne].copy(), edge_U=eU[:ne].copy(),
                fwd=fwd[:N].copy(), comp=comp[:N].copy(),
                stats={f: getattr(st, f) for f, _ in _Stats._fields_})


def count_threads(csr: OracleCSR, nthreads=1, stride=1, overlap=0.8, cutoffs=(1, 1, 0.66, 0.66, 0.66, 0.5),
                  qlen_diff=0.04, n_aln_diff=0.25):
    """CPU baseline: E* pair / edge counts over the query reads of every ``stride``-th 64-rank block,
    ``nthreads`` POSIX threads sharing one index (``fslr_oracle.c:oracle_count_threads``)."""
    L = lib()
    inp = _Input(csr.n_reads, *(_p(getattr(csr, f)) for f in ('read_off', 'chrom', 'start', 'end', 'aln', 'qlen2',
                                                               'nal', 'data_pos')))
    cut = np.ascontiguousarray(cutoffs, dtype=np.float64)
    prm = _Params(float(overlap), _p(cut), len(cut), float(qlen_diff), float(n_aln_diff), 10, 0, -1)
    st = _Stats()
    rc = L.oracle_count_threads(ctypes.byref(inp), ctypes.byref(prm), int(nthreads), int(stride), ctypes.byref(st))
    if rc == ORACLE_ZERO_DIVISION:
        raise OracleZeroDivision('division by zero')
    if rc != ORACLE_OK:
        raise RuntimeError(f'oracle_count_threads failed rc={rc}')
    return {f: getattr(st, f) for f, _ in _Stats._fields_}


def jaccard_lists(l1, l2, overlap):
    """KAT helper: ``l*`` = list of (chrom, start, end, aln); returns (I, U) or raises."""
    L = lib()
    a = np.array(l1, dtype=np.int64).reshape(-1, 4)
    b = np.array(l2, dtype=np.int64).reshape(-1, 4)
    cols = lambda m, k: np.ascontiguousarray(m[:, k])
    A = [cols(a, k) for k in range(4)]
    B = [cols(b, k) for k in range(4)]
    I = np.zeros(1, np.int64)
    U = np.zeros(1, np.int64)
    rc = L.oracle_jaccard_lists(len(a), *(_p(x) for x in A), len(b), *(_p(x) for x in B), float(overlap), _p(I),
                                _p(U))
    if rc == ORACLE_ZERO_DIVISION:
        raise OracleZeroDivision('division by zero')
    return int(I[0]), int(U[0])


def lengths_differ(q1, q2, n1, n2, qd, nd):
    out = np.zeros(1, np.int32)
    rc = lib().oracle_lengths_differ(int(q1), int(q2), int(n1), int(n2), float(qd), float(nd), _p(out))
    if rc == ORACLE_ZERO_DIVISION:
        raise OracleZeroDivision('division by zero')
    return bool(out[0])


# --------------------------------------------------------------------------------------
# host-stage restatement (plain loops; small inputs)
# --------------------------------------------------------------------------------------

def restate_mask_option(bed_chroms, cluster_mask_arg):
    """main.py:211-216: keep mask items that name a chromosome present in the bed, plus 'subtelomere'."""
    present = set(bed_chroms)
    out = set()
    if cluster_mask_arg:
        for item in cluster_mask_arg.split(','):
            if item == 'subtelomere' or item in present:
                out.add(item)
    return out


def restate_prep(bed, chrom_lengths, cluster_mask_arg='subtelomere', filter_false=False, threshold=500_000):
    """Return (OracleCSR with qnames by rank, bed_after_filter).

    ``bed`` is the DataFrame as read by ``pd.read_csv(..., sep='\\t')`` (main.py:209).
    """
    mask = restate_mask_option(bed['chrom'].tolist(), cluster_mask_arg)
    if filter_false:                                                   # cluster.py:80-86
        bed = bed[[('False' not in q) for q in bed['qname'].tolist()]]
    qn = bed['qname'].tolist()
    nrow = len(qn)
    # keep_fillings (cluster.py:14-31): drop the first and last row of every qname, file order
    first, last = {}, {}
    for r, q in enumerate(qn):
        first.setdefault(q, r)
        last[q] = r
    drop = set(first.values()) | set(last.values())
    keep_rows = [r for r in range(nrow) if r not in drop]
    qs = bed['qstart'].tolist()
    qe = bed['qend'].tolist()
    lo, hi = {}, {}
    for r in keep_rows:
        q = qn[r]
        lo[q] = qs[r] if q not in lo else min(lo[q], qs[r])
        hi[q] = qe[r] if q not in hi else max(hi[q], qe[r])
    # prepare_data (cluster.py:109-121): start/end = min/max(rstart, rend); pandas sort_values('start')
    # (quicksort argsort of the int64 column) defines `data` order
    rs = bed['rstart'].tolist()
    re_ = bed['rend'].tolist()
    chrom = bed['chrom'].tolist()
    aln = bed['aln_size'].tolist()
    nal = bed['n_alignments'].tolist()
    st = np.array([min(rs[r], re_[r]) for r in keep_rows], dtype=np.int64)
    order = st.argsort(kind='quicksort')
    # mask_sequences2 (cluster.py:89-106)
    long_chroms = {c: l for c, l in chrom_lengths.items() if l > 1_000_000}
    data = []
    for k in order:
        r = keep_rows[int(k)]
        c = chrom[r]
        s, e = min(rs[r], re_[r]), max(rs[r], re_[r])
        if mask:
            if c in mask:
                continue
            if 'subtelomere' in mask and c in long_chroms and (s < threshold or long_chroms[c] - e < threshold):
                continue
        data.append((c, s, e, aln[r], qn[r], nal[r], hi[qn[r]] - lo[qn[r]]))
    # ranks = first appearance in data (cluster.py:189-191); intervals per read in data order
    per_read = {}
    for pos, t in enumerate(data):
        per_read.setdefault(t[4], []).append((pos, t))
    chrom_id = {}
    names = list(per_read.keys())
    off = [0]
    cols = {k: [] for k in ('chrom', 'start', 'end', 'aln', 'qlen2', 'nal', 'data_pos')}
    for q in names:
        for pos, (c, s, e, a, _, n, q2) in per_read[q]:
            cols['chrom'].append(chrom_id.setdefault(c, len(chrom_id)))
            cols['start'].append(s)
            cols['end'].append(e)
            cols['aln'].append(a)
            cols['qlen2'].append(q2)
            cols['nal'].append(n)
            cols['data_pos'].append(pos)
        off.append(len(cols['start']))
    csr = OracleCSR(np.array(off), *(np.array(cols[k], dtype=np.int64) for k in
                                     ('chrom', 'start', 'end', 'aln', 'qlen2', 'nal', 'data_pos')), qnames=names)
    return csr, bed


def restate_numbering(bed_after_filter, csr: OracleCSR, comp: np.ndarray):
    """main.py:247-342 → dict qname → (cluster, n_reads) and the column dtype ('float'|'int').

    Returns ``None`` when the graph has no edges ("No clusters were found.").
    """
    comp = np.asarray(comp)
    if comp.size == 0 or comp.max() < 0:
        return None
    size = {}
    for c in comp.tolist():
        if c >= 0:
            size[c] = size.get(c, 0) + 1
    out = {}
    for r, c in enumerate(comp.tolist()):
        if c >= 0:
            out[csr.qnames[r]] = (c, size[c])
    k = max(size) + 1
    any_single = False
    for q in bed_after_filter['qname'].tolist():
        if q not in out:
            out[q] = (k, 1)
            k += 1
            any_single = True
    return out, ('float' if any_single else 'int')
