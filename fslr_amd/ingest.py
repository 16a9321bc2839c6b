"""Native reader for ``{name}.mappings.bed`` (C ABI ``include/fslr_ingest.h``).

Replaces ``pd.read_csv(f'{basename}.mappings.bed', sep='\\t')`` (reference ``fslr/main.py:209``)
for the columns the clustering path reads (``cluster.py:14`` keep_fillings, ``cluster.py:109``
prepare_data).  :func:`read_hot_columns` returns the frame
``pd.read_csv(path, sep='\\t', usecols=HOT_COLUMNS)`` would give, or ``None`` when the file is one
the fast path does not type exactly like pandas (quoted fields, NA spellings, non-canonical
integers, an all-integer string column); the caller then reads it with pandas.  Host code only:
this is the input side of the path, not the GPU product path.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
from ._lazy import pandas as pd

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'libfslr_ingest.so')
OK, ERROR, DECLINE = 0, 1, 2

INT_COLUMNS = ('rstart', 'rend', 'n_alignments', 'aln_size', 'qstart', 'qend')
STR_COLUMNS = ('chrom', 'qname')
HOT_COLUMNS = ('chrom', 'rstart', 'rend', 'qname', 'n_alignments', 'aln_size', 'qstart', 'qend')

_lib = None


class StaleLibrary(FileNotFoundError):
    """The reader library exists but was built from sources without an entry point this binding needs."""


def load(path: str = LIB_PATH):
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise FileNotFoundError(f'{path} is not built: run `make -C fslr_amd/csrc`')
    L = ctypes.CDLL(path)
    vp, i64, i32, cp = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_char_p
    sig = {
        'fslr_tsv_open': (i32, [cp, i32, ctypes.POINTER(vp), cp, ctypes.c_size_t]),
        'fslr_tsv_close': (None, [vp]),
        'fslr_tsv_rows': (i64, [vp]),
        'fslr_tsv_cols': (i32, [vp]),
        'fslr_tsv_colname': (cp, [vp, i32]),
        'fslr_tsv_find': (i32, [vp, cp]),
        'fslr_tsv_int_column': (i32, [vp, i32, vp]),
        'fslr_tsv_int_columns': (i32, [vp, i32, vp, vp]),
        'fslr_tsv_factorize': (i32, [vp, i32, vp, ctypes.POINTER(i64), ctypes.POINTER(i64)]),
        'fslr_tsv_uniques': (i32, [vp, i32, vp, vp]),
        'fslr_tsv_verbatim': (i32, [vp]),
        'fslr_tsv_scan': (i32, [vp, i32, vp, vp]),
        'fslr_tsv_scan_all': (i32, [vp, i32, vp, vp, i32, vp, vp, vp]),
        'fslr_tsv_write': (i32, [vp, cp, cp, vp, i64, vp, vp, vp, cp, ctypes.c_size_t]),
        'fslr_format_suffix': (i32, [i32, vp, vp, i64, vp, i64, vp]),
        'fslr_group_by_first_appearance': (i32, [vp, i64, i64, vp, vp, vp, vp]),
        'fslr_gather_i64': (i32, [i32, vp, vp, vp, i64, i32]),
        'fslr_argsort_distinct': (i32, [vp, i64, vp, i32]),
        'fslr_fillings': (i32, [i64, vp, i64, vp] + [vp] * 8 + [vp] + [vp] * 8 + [i32]),
    }
    missing = [name for name in sig if not hasattr(L, name)]
    if missing:
        # a library built from older sources: every caller treats it as not built (pandas / numpy)
        raise StaleLibrary(f'{path} lacks {", ".join(missing)}: rebuild it (make -C fslr_amd/csrc)')
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype, f.argtypes = res, args
    _lib = L
    return L


class TsvFile:
    """An opened, line-split TSV file (library-owned buffer)."""

    def __init__(self, path: str, n_threads: int = 0):
        L = load()
        err = ctypes.create_string_buffer(512)
        h = ctypes.c_void_p()
        rc = L.fslr_tsv_open(os.fsencode(path), int(n_threads), ctypes.byref(h), err, len(err))
        self.declined = rc == DECLINE
        if rc == ERROR:
            raise OSError(err.value.decode())
        self._h = h if rc == OK else None
        self._L = L

    def close(self):
        if self._h is not None:
            self._L.fslr_tsv_close(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    @property
    def rows(self) -> int:
        return int(self._L.fslr_tsv_rows(self._h))

    @property
    def columns(self) -> list:
        return [self._L.fslr_tsv_colname(self._h, i).decode() for i in range(self._L.fslr_tsv_cols(self._h))]

    def _col(self, name: str) -> int:
        c = self._L.fslr_tsv_find(self._h, name.encode())
        if c < 0:
            raise KeyError(name)
        return c

    def int_column(self, name: str):
        out = np.empty(self.rows, dtype=np.int64)
        rc = self._L.fslr_tsv_int_column(self._h, self._col(name), out.ctypes.data)
        return out if rc == OK else None

    def int_columns(self, names):
        """{name: int64[rows]} for several columns in one pass over the rows, or None."""
        names = list(dict.fromkeys(names))
        cols = np.asarray([self._col(n) for n in names], dtype=np.int32)
        outs = [np.empty(self.rows, dtype=np.int64) for _ in names]
        ptrs = (ctypes.c_void_p * len(outs))(*[o.ctypes.data for o in outs])
        rc = self._L.fslr_tsv_int_columns(self._h, len(names), cols.ctypes.data, ctypes.cast(ptrs, ctypes.c_void_p))
        return dict(zip(names, outs)) if rc == OK else None

    def factorize_codes(self, name: str):
        """(codes int32[rows], number of uniques) of ``pd.factorize(col, sort=False)``, or None; the
        uniques stay in the library until :meth:`uniques`."""
        c = self._col(name)
        codes = np.empty(self.rows, dtype=np.int32)
        nu, nb = ctypes.c_int64(), ctypes.c_int64()
        rc = self._L.fslr_tsv_factorize(self._h, c, codes.ctypes.data, ctypes.byref(nu), ctypes.byref(nb))
        if rc != OK:
            return None
        self._fact = getattr(self, '_fact', {})
        self._fact[name] = (int(nu.value), int(nb.value))
        return codes, int(nu.value)

    def uniques(self, name: str):
        """The uniques of the last :meth:`factorize_codes` of ``name`` (object array of str)."""
        nu, nb = self._fact[name]
        buf = np.empty(max(nb, 1), dtype=np.uint8)
        ends = np.empty(max(nu, 1), dtype=np.int64)
        self._L.fslr_tsv_uniques(self._h, self._col(name), buf.ctypes.data, ends.ctypes.data)
        raw = buf.tobytes()
        starts = np.concatenate(([0], ends[:nu - 1])) if nu else ends[:0]
        return np.array([raw[s:e].decode() for s, e in zip(starts.tolist(), ends[:nu].tolist())], dtype=object)

    def factorize(self, name: str):
        """(codes int32[rows], uniques object[k]) as ``pd.factorize(col, sort=False)``, or None."""
        f = self.factorize_codes(name)
        if f is None:
            return None
        return f[0], self.uniques(name)

    def scan(self, int_names):
        """verbatim() and int_columns(int_names) in one pass: the columns, or None when either fails."""
        names = list(dict.fromkeys(int_names))
        cols = np.asarray([self._col(n) for n in names], dtype=np.int32)
        outs = [np.empty(self.rows, dtype=np.int64) for _ in names]
        ptrs = (ctypes.c_void_p * len(outs))(*[o.ctypes.data for o in outs])
        rc = self._L.fslr_tsv_scan(self._h, len(names), cols.ctypes.data, ctypes.cast(ptrs, ctypes.c_void_p))
        return dict(zip(names, outs)) if rc == OK else None

    def scan_all(self, int_names, str_names):
        """scan() that also factorizes ``str_names`` in the same pass: ({name: int64[rows]},
        {name: (codes int32[rows], number of uniques)}), or None.  :meth:`uniques` gives the values."""
        names = list(dict.fromkeys(int_names))
        snames = list(dict.fromkeys(str_names))
        cols = np.asarray([self._col(n) for n in names], dtype=np.int32)
        scols = np.asarray([self._col(n) for n in snames], dtype=np.int32)
        outs = [np.empty(self.rows, dtype=np.int64) for _ in names]
        codes = [np.empty(self.rows, dtype=np.int32) for _ in snames]
        counts = np.zeros(2 * max(1, len(snames)), dtype=np.int64)
        ptrs = (ctypes.c_void_p * max(1, len(outs)))(*[o.ctypes.data for o in outs])
        sptrs = (ctypes.c_void_p * max(1, len(codes)))(*[o.ctypes.data for o in codes])
        rc = self._L.fslr_tsv_scan_all(self._h, len(names), cols.ctypes.data, ctypes.cast(ptrs, ctypes.c_void_p),
                                       len(snames), scols.ctypes.data, ctypes.cast(sptrs, ctypes.c_void_p),
                                       counts.ctypes.data)
        if rc != OK:
            return None
        self._fact = getattr(self, '_fact', {})
        strs = {}
        for k, n in enumerate(snames):
            self._fact[n] = (int(counts[2 * k]), int(counts[2 * k + 1]))
            strs[n] = (codes[k], int(counts[2 * k]))
        return dict(zip(names, outs)), strs

    def verbatim(self) -> bool:
        return self._L.fslr_tsv_verbatim(self._h) == OK

    def write_rows(self, path: str, rows, suffix_frame: pd.DataFrame, suffix_key) -> None:
        """Write input rows ``rows`` + the columns of ``suffix_frame`` like ``DataFrame.to_csv``.

        ``suffix_frame`` is constant per ``suffix_key`` value (one value per output row); pandas
        formats one row per distinct key, so the appended numbers are pandas' own text.
        ``suffix_key``: a Series / array of keys, or ``(codes, uniques)`` already factorized.
        """
        rows = np.ascontiguousarray(rows, dtype=np.int64)
        if isinstance(suffix_key, tuple):
            codes, uniq = suffix_key
        else:
            codes, uniq = pd.factorize(suffix_key, sort=False)
        first = np.full(len(uniq), -1, dtype=np.int64)
        first[codes[::-1]] = np.arange(len(codes) - 1, -1, -1)
        per_key = suffix_frame.iloc[first]
        got = format_suffix(per_key)
        if got is not None:
            buf, ends = got
        else:
            text = per_key.to_csv(sep='\t', header=False, index=False, lineterminator='\n')
            lines = text.split('\n')[:len(uniq)]
            enc = [('\t' + ln).encode() for ln in lines]
            ends = np.cumsum([len(x) for x in enc], dtype=np.int64) if enc else np.zeros(1, np.int64)
            buf = b''.join(enc) or b'\0'
        head = ''.join('\t' + str(c) for c in suffix_frame.columns).encode()
        sid = np.ascontiguousarray(codes, dtype=np.int32)
        err = ctypes.create_string_buffer(512)
        rc = self._L.fslr_tsv_write(self._h, os.fsencode(path), head, rows.ctypes.data, len(rows), sid.ctypes.data,
                                    buf, ends.ctypes.data, err, len(err))
        if rc != OK:
            raise OSError(err.value.decode())


def format_suffix(frame: pd.DataFrame):
    """(buffer, ends) of ``frame.to_csv(sep='\\t', header=False, index=False)``'s rows, each prefixed
    by a tab, formatted natively (fslr_format_suffix) for int64 / finite float64 columns, or None
    (the caller formats with pandas)."""
    L = load()
    n = len(frame)
    kinds, arrs = [], []
    for c in frame.columns:
        v = frame[c].to_numpy()
        if v.dtype == np.int64:
            kinds.append(0)
        elif v.dtype == np.float64:
            kinds.append(1)
        else:
            return None
        arrs.append(np.ascontiguousarray(v))
    if not arrs or n == 0:
        return None
    cap = n * len(arrs) * 40 + 16
    out = np.empty(cap, dtype=np.uint8)
    ends = np.empty(n, dtype=np.int64)
    k = np.asarray(kinds, dtype=np.int32)
    ptrs = (ctypes.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])
    rc = L.fslr_format_suffix(len(arrs), k.ctypes.data, ctypes.cast(ptrs, ctypes.c_void_p), n, out.ctypes.data, cap,
                              ends.ctypes.data)
    if rc != OK:
        return None
    return out[:int(ends[-1])].tobytes() or b'\0', ends


def group_by_first_appearance(codes):
    """(read_code, off, perm) of the codes grouped by first appearance (fslr_group_by_first_appearance),
    or None when the codes are not small non-negative ints or the library is not built."""
    c = np.ascontiguousarray(codes, dtype=np.int64)
    n = c.size
    if n == 0 or c.min() < 0 or c.max() >= 4 * n + 1024:
        return None
    try:
        L = load()
    except FileNotFoundError:
        return None
    read_code = np.empty(n, dtype=np.int64)
    off = np.empty(n + 1, dtype=np.int64)
    perm = np.empty(n, dtype=np.int64)
    nr = ctypes.c_int64()
    rc = L.fslr_group_by_first_appearance(c.ctypes.data, n, int(c.max()) + 1, read_code.ctypes.data,
                                          ctypes.byref(nr), off.ctypes.data, perm.ctypes.data)
    if rc != OK:
        return None
    return read_code[:nr.value], off[:nr.value + 1], perm


def gather_columns(columns, idx, n_threads: int = 0):
    """[c[idx] for c in columns] as int64, in one threaded native pass (fslr_gather_i64); numpy when
    the library is not built.  ``idx`` must index every column in range."""
    idx = np.ascontiguousarray(idx, dtype=np.int64)
    src = [np.ascontiguousarray(c, dtype=np.int64) for c in columns]
    try:
        L = load()
    except FileNotFoundError:
        return [c[idx] for c in src]
    out = [np.empty(idx.size, dtype=np.int64) for _ in src]
    sp = (ctypes.c_void_p * len(src))(*[c.ctypes.data for c in src])
    dp = (ctypes.c_void_p * len(out))(*[o.ctypes.data for o in out])
    rc = L.fslr_gather_i64(len(src), ctypes.cast(sp, ctypes.c_void_p), ctypes.cast(dp, ctypes.c_void_p),
                           idx.ctypes.data, idx.size, int(n_threads))
    if rc != OK:
        raise RuntimeError('fslr_gather_i64 failed')
    return out


def argsort_distinct(keys, n_threads: int = 0):
    """The argsort of ``keys`` when no two keys tie (then every sort agrees, numpy's quicksort
    included), by a threaded native radix sort; None when two keys tie, the key range is wider
    than 2^32 or the library is not built (the caller sorts with numpy)."""
    keys = np.ascontiguousarray(keys, dtype=np.int64)
    try:
        L = load()
    except FileNotFoundError:
        return None
    order = np.empty(keys.size, dtype=np.int64)
    rc = L.fslr_argsort_distinct(keys.ctypes.data, keys.size, order.ctypes.data, int(n_threads))
    return order if rc == 1 else None


class QnameCodes:
    """``pd.factorize(qname, sort=False)`` of a file's rows, made by the reader.  Frames derived
    from the read frame carry it in ``attrs`` (shared, never copied: pandas deep-copies attrs), so
    the clustering block does not hash 10M qname strings once per stage; :func:`factorize_qname`
    takes the rows a derived frame kept by its index (the file's row numbers)."""

    def __init__(self, codes, uniq):
        self.codes = codes
        self.uniq = uniq

    def __deepcopy__(self, memo):
        return self

    def __copy__(self):
        return self


ATTR = 'fslr_qname_codes'


def factorize_qname(df: pd.DataFrame):
    """``pd.factorize(df['qname'], sort=False)``: codes in first-appearance order and the uniques.

    From the reader's codes when ``df`` came from :func:`frame_from` (its rows are file rows, its
    index their row numbers, its qname column unchanged); otherwise by pandas."""
    qc = df.attrs.get(ATTR)
    if not isinstance(qc, QnameCodes):
        return pd.factorize(df['qname'], sort=False)
    idx = df.index
    if isinstance(idx, pd.RangeIndex) and idx.start == 0 and idx.step == 1 and len(idx) == len(qc.codes):
        return qc.codes, qc.uniq
    c = qc.codes[idx.to_numpy()]
    n_u = len(qc.uniq)
    first = np.full(n_u, -1, dtype=np.int64)
    first[c[::-1]] = np.arange(len(c) - 1, -1, -1)          # first row of each code present
    present = np.flatnonzero(first >= 0)
    order = present[np.argsort(first[present], kind='stable')]
    remap = np.full(n_u, -1, dtype=np.int64)
    remap[order] = np.arange(order.size)
    return remap[c], qc.uniq[order]


def frame_from(t: 'TsvFile', int_columns=INT_COLUMNS, str_columns=STR_COLUMNS):
    """The columns (file order) as pandas would type them, or None.  The qname codes ride along
    in ``attrs`` (:class:`QnameCodes`)."""
    if t.declined or not (set(int_columns) | set(str_columns)) <= set(t.columns):
        return None
    cols = t.int_columns([c for c in int_columns if c not in str_columns])
    if cols is None:
        return None
    qcodes = None
    for name in str_columns:
        f = t.factorize(name)
        if f is None:
            return None
        cols[name] = f[1][f[0]]
        if name == 'qname':
            qcodes = QnameCodes(f[0], f[1])
    df = pd.DataFrame({c: cols[c] for c in t.columns if c in cols})
    if qcodes is not None:
        df.attrs[ATTR] = qcodes
    return df


def read_hot_columns(path: str, n_threads: int = 0):
    """``pd.read_csv(path, sep='\\t', usecols=HOT_COLUMNS)`` natively, or None (read with pandas)."""
    with TsvFile(path, n_threads) as t:
        return frame_from(t)


def fillings(qcode, n_q, row_keep, ints, ccode, chrom_lut, n_threads: int = 0):
    """keep_fillings + prepare_data's per-row columns natively (fslr_fillings): a dict of int64 columns
    frow, start, end, aln, qcode, nal, qlen2, chrom over the fillings in file order."""
    L = load()
    n = int(qcode.shape[0])
    qcode = np.ascontiguousarray(qcode, np.int32)
    ccode = np.ascontiguousarray(ccode, np.int32)
    lut = np.ascontiguousarray(chrom_lut, np.int64)
    keep = None if row_keep is None else np.ascontiguousarray(row_keep, np.uint8)
    src = [np.ascontiguousarray(ints[k], np.int64) for k in ('rstart', 'rend', 'aln_size', 'qstart', 'qend',
                                                                'n_alignments')]
    names = ('frow', 'start', 'end', 'aln', 'qcode', 'nal', 'qlen2', 'chrom')
    out = {k: np.empty(n, np.int64) for k in names}
    n_out = ctypes.c_int64()
    rc = L.fslr_fillings(n, qcode.ctypes.data, int(n_q), keep.ctypes.data if keep is not None else None,
                         *(a.ctypes.data for a in src), ccode.ctypes.data, lut.ctypes.data, ctypes.byref(n_out),
                         *(out[k].ctypes.data for k in names), int(n_threads))
    if rc != OK:
        raise RuntimeError('fslr_fillings failed')
    m = int(n_out.value)
    return {k: v[:m] for k, v in out.items()}

