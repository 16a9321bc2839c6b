"""The clustering block of ``fslr --skip-alignment`` on columns (reference ``fslr/main.py:190-352``).

``main.run_clustering`` takes this path when the native reader accepts the input (every column
round-trips through pandas unchanged, ``ingest.TsvFile.verbatim``) and ``--filter-high-coverage``
is off.  It computes what the pandas path computes — rename_chromosomes, delete_false,
keep_fillings, prepare_data (cluster.py:14-121), the device query, assign_clusters
(main.py:251-342) and choose_alignment (cluster.py:237-254) — on int64 columns and the reader's
qname / chrom codes, never on a frame of rows or on qname strings, and writes the outputs as the
input's own row bytes plus the appended columns (the native writer), byte-identical to
``DataFrame.to_csv`` of the pandas path.  The GPU CLI tests compare both paths with the
reference's outputs on every fixture.

Codes: ``qcode[row]`` numbers qnames by first appearance in the file (pd.factorize order).  Rows
removed by delete_false remove whole qnames, so the first-appearance order of the qnames left is
still ascending code order — what assign_clusters' singleton numbering and the writers' per-qname
suffixes rely on.
"""
from __future__ import annotations

import ctypes
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

from . import cluster, ingest
from ._lib import FSLR_MAX_L, FslrError
from .prep import IntervalData, data_order, mask_keep

INT_COLS = ('rstart', 'rend', 'n_alignments', 'aln_size', 'qstart', 'qend', 'alignment_score')
STR_COLS = ('qname', 'chrom')


class Fallback(Exception):
    """The input needs the pandas path (a case the columns do not reproduce exactly)."""


def chrom_map(names):
    """rename_chromosomes' numbering (cluster.rename_chromosomes) of first-appearance chrom names."""
    order = sorted(range(len(names)), key=lambda i: (cluster._chrom_key(names[i]), i))
    return {names[i]: k + 1 for k, i in enumerate(order)}


def _suffix(cols):
    """(buffer, ends) of the tab-prefixed text DataFrame.to_csv writes for per-key int64 / float64
    columns (ingest.format_suffix's native formatter)."""
    L = ingest.load()
    n = len(cols[0])
    kinds = np.asarray([0 if c.dtype == np.int64 else 1 for c in cols], dtype=np.int32)
    arrs = [np.ascontiguousarray(c) for c in cols]
    if n == 0:
        return b'\0', np.zeros(1, np.int64)
    cap = n * len(arrs) * 40 + 16
    out = np.empty(cap, dtype=np.uint8)
    ends = np.empty(n, dtype=np.int64)
    ptrs = (ctypes.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])
    rc = L.fslr_format_suffix(len(arrs), kinds.ctypes.data, ctypes.cast(ptrs, ctypes.c_void_p), n, out.ctypes.data,
                              cap, ends.ctypes.data)
    if rc != ingest.OK:
        raise Fallback('suffix formatting')
    return out[:int(ends[-1])].tobytes() or b'\0', ends


def _write(tsv, path, rows, key_of_row, names, cols):
    """Rows ``rows`` of the input, each followed by the per-key values ``cols`` (key_of_row[k])."""
    buf, ends = _suffix(cols)
    head = ''.join('\t' + n for n in names).encode()
    rows = np.ascontiguousarray(rows, dtype=np.int64)
    sid = np.ascontiguousarray(key_of_row, dtype=np.int32)
    err = ctypes.create_string_buffer(512)
    rc = tsv._L.fslr_tsv_write(tsv._h, path.encode(), head, rows.ctypes.data, len(rows), sid.ctypes.data, buf,
                               ends.ctypes.data, err, len(err))
    if rc != ingest.OK:
        raise OSError(err.value.decode())


def run(args, basename, tsv, ints, strs, t):
    """main.py:190-352 on columns (``ints``: INT_COLS of every row, ``strs``: the STR_COLS codes, both
    from TsvFile.scan_all); returns False for "No clusters were found." (as the pandas path), True
    after writing both outputs.  Raises Fallback before writing anything when a step needs the
    pandas path; the HIP context it opened is closed first, so the pandas path opens the only one."""
    # the HIP context comes up while the host prepares the input (one GPU; the multi-GPU ranks make
    # their own)
    pool = ThreadPoolExecutor(3)
    ctx_f = pool.submit(cluster._open_context, args.get('device')) if (args.get('gpus') or 1) == 1 else None
    state = {'trees': None}
    try:
        return _run(args, basename, tsv, ints, strs, t, pool, ctx_f, state)
    except BaseException:
        pool.shutdown(wait=True)
        ctx = state['trees'].ctx if state['trees'] is not None and hasattr(state['trees'], 'ctx') else None
        if ctx is None and ctx_f is not None and ctx_f.done() and ctx_f.exception() is None:
            ctx = ctx_f.result()
        if ctx is not None:
            ctx.close()
        raise


def _run(args, basename, tsv, ints, strs, t, pool, ctx_f, state):
    t1 = time.perf_counter()
    n_rows = tsv.rows
    qcode, n_q = strs['qname']
    ccode, _ = strs['chrom']
    chrom_names = list(tsv.uniques('chrom'))
    score = ints['alignment_score']
    if n_rows and np.abs(score).max() >= (1 << 53) // max(1, n_rows):
        raise Fallback('alignment_score range')          # choose_alignment's exact-mean argument
    t['read_csv'] += time.perf_counter() - t1

    t1 = time.perf_counter()
    # main.py:199-206 cluster mask; cluster.py:34-43 rename_chromosomes
    mask_names = set()
    if args['cluster_mask']:
        allowed = set(chrom_names)
        for item in args['cluster_mask'].split(','):
            if item in allowed or item == 'subtelomere':
                mask_names.add(item)
    lens = cluster.get_chromosome_lengths(f'{basename}.bwa_dodi.bam')
    cmap = chrom_map(chrom_names)
    chr_lengths = {cmap.get(k): v for k, v in lens.items()}
    mask = [cmap.get(x) if x != 'subtelomere' else x for x in mask_names]
    chrom_num = np.asarray([cmap[c] for c in chrom_names], dtype=np.int64)
    # cluster.py:80-86 delete_false: whole qnames go
    row_keep = None
    if args['filter_false']:
        bad_q = np.fromiter(('False' in q for q in tsv.uniques('qname')), dtype=bool, count=n_q)
        row_keep = ~bad_q[qcode]
        rows = np.flatnonzero(row_keep)
    else:
        rows = np.arange(n_rows, dtype=np.int64)
    # cluster.py:14-31 keep_fillings (each qname's first and last row dropped, qlen2 = its fillings'
    # span) and cluster.py:109-121 prepare_data's columns (min/max of rstart/rend), natively
    f = ingest.fillings(qcode, n_q, row_keep, ints, ccode, chrom_num)
    start = f['start']
    t['prepare.fill'] = time.perf_counter() - t1
    # prepare_data's sort_values('start') (pandas' quicksort argsort, ties included; numpy sorts
    # without the GIL, so mask_sequences2, the writers' per-qname sums and the rows' upload to the
    # device run beside it)
    order_f = pool.submit(data_order, start)
    rows_f = pool.submit(_rows_upload, ctx_f, f, n_q, int(chrom_num.max(initial=0)) + 1) \
        if ctx_f is not None and start.size else None
    keepm = mask_keep(f['chrom'], start, f['end'], mask, chr_lengths, 500_000) if mask else None
    qc = qcode[rows].astype(np.int64)
    w = _writer_prep(qc, n_q, score[rows])
    order = order_f.result()
    t['prepare.sort'] = time.perf_counter() - t1 - t['prepare.fill']

    def host_data():
        # the prepared `data` list as columns on the host (IntervalData): the masked order's gathers
        o = order if keepm is None else order[keepm[order]]
        c, s, e, a, q, nal, ql2, ix = ingest.gather_columns([f['chrom'], start, f['end'], f['aln'], f['qcode'],
                                                             f['nal'], f['qlen2'], f['frow']], o)
        return IntervalData(chrom=c, start=s, end=e, aln_size=a, qcode=q, qnames=_LazyQnames(tsv, n_q),
                            n_alignments=nal, qlen2=ql2, middle=a // 2 + s, index=ix)
    trees = None
    if rows_f is not None and rows_f.result():
        # the device makes the `data` list, the read ranks and the CSR from the rows (fslr_set_reads_rows)
        ctx = ctx_f.result()
        t['prepare'] = time.perf_counter() - t1
        t1 = time.perf_counter()
        try:
            info = ctx.set_reads_rows(order, keepm, args['overlap'])
        except FslrError as e:
            if getattr(e, 'info', {}).get('max_len', 0) <= FSLR_MAX_L:
                raise
            info = None                          # reads of more than FSLR_MAX_L intervals: the host CSR
        if info is not None:
            data = _LazyData(host_data)
            csr = cluster.RowsCSR(ctx, info)
            t['csr'] = time.perf_counter() - t1
            t2 = time.perf_counter()
            trees = state['trees'] = cluster.RowsIndex(data, csr, ctx, args['overlap'])
            pool.shutdown()
            t['upload'] = time.perf_counter() - t2
    if trees is None:
        data = host_data()
        t['prepare'] = time.perf_counter() - t1
        t1 = time.perf_counter()
        csr = data.csr()
        t['csr'] = time.perf_counter() - t1
        t2 = time.perf_counter()
        trees = state['trees'] = cluster.build_interval_trees(data, device=args.get('device'),
                                                              n_gpus=args.get('gpus') or 1,
                                                              ctx=ctx_f.result() if ctx_f is not None else None)
        pool.shutdown()
        t['upload'] = time.perf_counter() - t2
    t2 = time.perf_counter()
    g = cluster.query_graph(trees, data, args['overlap'], [float(i) for i in args['jaccard_cutoffs'].split(',')], 10,
                            args['qlen_diff'], args['n_alignment_diff'])
    t['query'] = time.perf_counter() - t2
    if g.n_edges == 0:
        print('No clusters were found.')
        return False

    t3 = time.perf_counter()
    # main.py:251-342 assign_clusters: components by min rank (networkx order), then the qnames
    # without an edge in first-appearance order, n_reads 1; float columns when any such qname
    lab = g.labels
    nr = lab.shape[0]
    sizes = np.bincount(lab, minlength=nr)
    roots = np.flatnonzero(sizes >= 2)
    rid = np.full(nr, -1, np.int64)
    rid[roots] = np.arange(roots.size)
    node = sizes[lab] >= 2
    q_cid = np.full(n_q, -1, np.int64)
    q_size = np.zeros(n_q, np.int64)
    rq = csr.read_qcode[node]
    q_cid[rq] = rid[lab[node]]
    q_size[rq] = sizes[lab[node]]
    present, keys, key_of_code, avg, first_row = w
    single = present & (q_cid < 0)
    k = int(single.sum())
    q_cid[single] = roots.size + np.arange(k)
    q_size[single] = 1
    cl_k, nr_k = q_cid[keys], q_size[keys]
    if k:
        cl_k, nr_k = cl_k.astype(np.float64), nr_k.astype(np.float64)
    t['write.assign'] = time.perf_counter() - t3
    # the two files are written at once (each by its own native writer threads; ctypes releases the
    # GIL): the representative rows are chosen while the cluster file is being written
    wpool = ThreadPoolExecutor(2)
    try:
        fut_c = wpool.submit(_write, tsv, f'{basename}.mappings.cluster.bed', rows, key_of_code[qc],
                             ['cluster', 'n_reads'], [cl_k, nr_k])
        # cluster.py:237-254 choose_alignment: per cluster the qname with the highest mean score, the
        # first in file order on ties; its rows
        cid_k = q_cid[keys]
        best = np.full(int(cid_k.max()) + 1, -np.inf)
        np.maximum.at(best, cid_k, avg[keys])
        cand = keys[avg[keys] == best[cid_k]]
        win = np.full(best.size, rows.size, np.int64)
        np.minimum.at(win, q_cid[cand], first_row[cand])
        chosen = np.zeros(n_q, bool)
        chosen[qc[win[win < rows.size]]] = True
        rsel = chosen[qc]
        t['write.choose'] = time.perf_counter() - t3 - t['write.assign']
        fut_r = wpool.submit(_write, tsv, f'{basename}.mappings.representative.bed', rows[rsel], key_of_code[qc[rsel]],
                             ['cluster', 'n_reads', 'avg_alignment_score'], [cl_k, nr_k, avg[keys]])
        fut_c.result()
        t['write.cluster'] = time.perf_counter() - t3 - t['write.assign']
        fut_r.result()
    finally:
        wpool.shutdown(wait=True)
    t['write'] = time.perf_counter() - t3
    # the device buffers go now (the caller's process would free them at exit anyway)
    t5 = time.perf_counter()
    ctx = getattr(trees, 'ctx', None)
    if ctx is not None and hasattr(ctx, 'close'):
        ctx.close()
    t['close'] = time.perf_counter() - t5
    if args.get('timings'):
        st = g.stats
        import sys
        print('timings_s ' + ' '.join(f'{k}={v:.3f}' for k, v in t.items()) +
              f' evaluated_pairs={st.get("evaluated_pairs", -1)} edges={g.n_edges} max_fwd={st.get("max_fwd", -1)}'
              ' path=columns', file=sys.stderr)
    return True


def _writer_prep(qc, n_q, score):
    """What the writers need that does not depend on the graph: the qnames present (ascending code =
    first-appearance order) and their key numbers, each qname's mean alignment_score
    (choose_alignment's groupby mean: a float64 sum of int64 values below 2**53 is exact in any
    order) and its first row."""
    present = np.zeros(n_q, bool)
    present[qc] = True
    keys = np.flatnonzero(present)
    key_of_code = np.full(n_q, -1, np.int64)
    key_of_code[keys] = np.arange(keys.size)
    sums = np.bincount(qc, weights=score.astype(np.float64), minlength=n_q)
    cnt = np.bincount(qc, minlength=n_q)
    with np.errstate(invalid='ignore', divide='ignore'):
        avg = sums / cnt
    first_row = np.full(n_q, qc.size, np.int64)
    st = _run_starts(qc)
    if st is not None:
        first_row[qc[st]] = st
    else:
        np.minimum.at(first_row, qc, np.arange(qc.size))
    return present, keys, key_of_code, avg, first_row


def _run_starts(codes):
    """Start of each run of equal codes when every code's rows form one run (a qname-grouped file, as
    the mapping step writes it), else None."""
    if codes.size == 0:
        return np.zeros(0, np.int64)
    st = np.concatenate(([0], np.flatnonzero(codes[1:] != codes[:-1]) + 1))
    distinct = np.count_nonzero(np.bincount(codes))
    return st if distinct == st.size else None


def _rows_upload(ctx_f, f, n_q, n_chrom_ids):
    """The fillings' columns to the device (fslr_rows_upload) while the host sorts; False when no
    context came up (the CPU tests stand the oracle in for the device)."""
    ctx = ctx_f.result()
    if ctx is None:
        return False
    ctx.rows_upload(f, n_q, n_chrom_ids)
    return True


class _LazyData:
    """IntervalData of the device path: built on the host only if something reads it."""

    def __init__(self, build):
        self._build, self._d = build, None

    def _get(self):
        if self._d is None:
            self._d = self._build()
        return self._d

    def __len__(self):
        return len(self._get())

    def __getattr__(self, name):
        if name.startswith('_'):
            raise AttributeError(name)
        return getattr(self._get(), name)


class _LazyQnames:
    """IntervalData.qnames for the columnar path: decoded from the reader only if indexed."""

    def __init__(self, tsv, n):
        self._tsv, self._n, self._u = tsv, n, None

    def __len__(self):
        return self._n

    def __getitem__(self, k):
        if self._u is None:
            self._u = self._tsv.uniques('qname')
        return self._u[k]


__all__ = ['run', 'Fallback', 'chrom_map']
