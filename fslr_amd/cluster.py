"""Drop-in replacement of ``fslr/cluster.py`` whose hot path runs on MI355X.

Same function names, arguments and return shapes as the reference module
(/root/reference/fslr/cluster.py); the per-pair work of ``query_interval_trees``
and the connected components run in ``libfslr_hip.so`` (HIP, gfx950).  Host
stages are vectorised numpy/pandas with the reference's exact semantics.

Function map (reference file:line → here):
  keep_fillings              cluster.py:14-31    vectorised first/last drop + group span
  rename_chromosomes         cluster.py:34-43    chrN by N, others after (equality-only downstream)
  chrom_to_str               cluster.py:46-49
  calc_coverage              cluster.py:52-67
  filter_high_coverage       cluster.py:70-77
  delete_false               cluster.py:80-86
  mask_sequences2            cluster.py:89-106   vectorised for IntervalData
  prepare_data               cluster.py:109-121  → IntervalData (sequence of IntervalItem)
  build_interval_trees       cluster.py:124-130  → DeviceIntervalIndex (HBM CSR + sorted index)
  get_chromosome_lengths     cluster.py:173-175  own BGZF/BAM header reader (no pysam)
  query_interval_trees       cluster.py:187-227  device pair kernel; returns (match_df, ClusterGraph)
  get_subgraphs              cluster.py:230-234  components ordered by min read rank
  choose_alignment           cluster.py:237-254  vectorised groupby/idxmax
"""
from __future__ import annotations

import os
import sys
import warnings

import numpy as np
from ._lazy import pandas as pd

from . import bam_header, ingest, multi
from ._lib import FSLR_MAX_L, FSLR_THR_ZERO_ALN, Context
from .prep import (CSR, IntervalData, IntervalItem, build_csr, data_order, first_last_masks, fold_overlap_threshold,
                   group_span, has_long_reads, mask_keep, pass_table, umax_table)

__all__ = ['IntervalItem', 'keep_fillings', 'rename_chromosomes', 'chrom_to_str', 'calc_coverage',
           'filter_high_coverage', 'delete_false', 'mask_sequences2', 'prepare_data', 'build_interval_trees',
           'get_chromosome_lengths', 'query_interval_trees', 'get_subgraphs', 'choose_alignment',
           'ClusterGraph', 'DeviceIntervalIndex', 'MultiGpuIndex', 'EdgeCapWarning']


class EdgeCapWarning(UserWarning):
    """The reference's result depends on an order this build cannot pin: n_alignments
    that differ between rows of one read (cluster.py:209 reads the row its search
    reaches first)."""


def _default_device() -> int:
    return int(os.environ.get('FSLR_DEVICE', os.environ.get('LOCAL_RANK', '0')))


# ------------------------------------------------------------------ host stages
def keep_fillings(bed_file: pd.DataFrame) -> pd.DataFrame:
    """cluster.py:14-31: drop the first and last row (file order) of every qname; add qlen2."""
    codes, uniq = ingest.factorize_qname(bed_file)
    first, last = first_last_masks(codes)
    keep = ~(first | last)
    out = bed_file[keep]
    kc = codes[keep]
    span = group_span(kc, out['qstart'].to_numpy(), out['qend'].to_numpy(), len(uniq))
    with warnings.catch_warnings():
        warnings.simplefilter('ignore')
        out['qlen2'] = span[kc]
    return out


def _chrom_key(name):
    if isinstance(name, str) and name[:3] == 'chr' and name[3:].isdigit():
        return (0, int(name[3:]))
    return (1, 0)


def rename_chromosomes(bed_file, chromosome_lengths, chromosome_mask):
    """cluster.py:34-43.  chrN → N-order ids, other names after (first-appearance order).

    Only equality of ids is used downstream, so this deterministic numbering is
    interchangeable with the reference's set-iteration order for non-chrN names.
    """
    names = list(pd.unique(bed_file['chrom']))
    order = sorted(range(len(names)), key=lambda i: (_chrom_key(names[i]), i))
    cmap = {names[i]: k + 1 for k, i in enumerate(order)}
    chr_lengths = {cmap.get(k): v for k, v in chromosome_lengths.items()}
    bed_file['chrom'] = bed_file['chrom'].map(cmap)
    mask = [cmap.get(x) if x != 'subtelomere' else x for x in chromosome_mask]
    return bed_file, chr_lengths, mask, cmap


def chrom_to_str(bed_df, chromosome_to_numeric_map):
    """cluster.py:46-49."""
    inv = {v: k for k, v in chromosome_to_numeric_map.items()}
    bed_df['chrom'] = bed_df['chrom'].map(inv)
    return bed_df


def calc_coverage(bed_file, chromosome_lengths):
    """cluster.py:52-67: per-chromosome +1/-1 coverage at rstart/rend, cumulative."""
    cov = {}
    for chrom, grp in bed_file.groupby('chrom'):
        if chrom not in chromosome_lengths:
            continue
        c = np.zeros(chromosome_lengths[chrom] + 1)
        np.add.at(c, grp['rstart'].to_numpy(), 1)
        np.add.at(c, grp['rend'].to_numpy(), -1)
        cov[chrom] = np.cumsum(c)
    return cov


def filter_high_coverage(data, bed_file, chromosome_lengths, threshold):
    """cluster.py:70-77.  (main.py:235 passes a DataFrame here, which fails in the
    reference exactly as it fails here: iterating a DataFrame yields column names.)"""
    cov = calc_coverage(bed_file, chromosome_lengths)
    if isinstance(data, IntervalData):
        keep = np.array([cov[c][m] <= threshold for c, m in zip(data.chrom.tolist(), data.middle.tolist())],
                        dtype=bool)
        return data.select(keep)
    return [aln for aln in data if not cov[aln.chrom][aln.middle] > threshold]


def delete_false(bed_file):
    """cluster.py:80-86."""
    return bed_file[~bed_file['qname'].str.contains('False')]


def mask_sequences2(read_alignments, mask, chromosome_lengths, threshold=500_000):
    """cluster.py:89-106 (lines 104-105 can never fire: len==1 and >=4)."""
    if not mask:
        return read_alignments
    if isinstance(read_alignments, IntervalData):
        keep = mask_keep(read_alignments.chrom, read_alignments.start, read_alignments.end, mask,
                         chromosome_lengths, threshold)
        return read_alignments.select(keep)
    long_ = {k: v for k, v in chromosome_lengths.items() if v > 1_000_000}
    out = []
    for a in read_alignments:
        if a.chrom in mask:
            continue
        if 'subtelomere' in mask and a.chrom in long_ and (a.start < threshold or long_[a.chrom] - a.end < threshold):
            continue
        out.append(a)
    return out


def prepare_data(bed_df, cluster_mask, chromosome_lengths, threshold=500_000) -> IntervalData:
    """cluster.py:109-121 → IntervalData in ``sort_values('start')`` order, masked."""
    rs = bed_df['rstart'].to_numpy()
    re_ = bed_df['rend'].to_numpy()
    start = np.minimum(rs, re_)
    end = np.maximum(rs, re_)
    aln = bed_df['aln_size'].to_numpy()
    with warnings.catch_warnings():
        warnings.simplefilter('ignore')
        bed_df['start'] = start
        bed_df['end'] = end
        bed_df['middle'] = aln // 2 + start
    order = data_order(start)
    codes, uniq = ingest.factorize_qname(bed_df)
    chrom = bed_df['chrom'].to_numpy()
    if chrom.dtype.kind not in 'iu':                    # not renamed (rename_chromosomes not called)
        chrom = pd.factorize(bed_df['chrom'], sort=False)[0]
    if cluster_mask:
        # mask_sequences2 (cluster.py:89-106) is a per-interval predicate applied to the sorted list:
        # evaluated before the sort, one gather does both
        keep = mask_keep(np.asarray(chrom, np.int64), np.asarray(start, np.int64), np.asarray(end, np.int64),
                         cluster_mask, chromosome_lengths, threshold)
        order = order[keep[order]]
    cols = ingest.gather_columns([chrom, start, end, aln, codes, bed_df['n_alignments'].to_numpy(),
                                  bed_df['qlen2'].to_numpy(), aln // 2 + start], order)
    c, s, e, a, q, nal, ql2, mid = cols
    ix = bed_df.index.to_numpy()[order]
    return IntervalData(chrom=c, start=s, end=e, aln_size=a, qcode=q, qnames=np.asarray(uniq, dtype=object),
                        n_alignments=nal, qlen2=ql2, middle=mid, index=ix)


def get_chromosome_lengths(bam_path):
    """cluster.py:173-175 (BAM header reference dictionary)."""
    return bam_header.get_chromosome_lengths(bam_path)


# ------------------------------------------------------------------ device stages
class DeviceIntervalIndex:
    """What build_interval_trees returns: the CSR in HBM plus the sorted interval index."""

    def __init__(self, data, device: int | None = None, ctx: Context | None = None):
        self.source = data                      # what the caller passed (query_interval_trees checks it)
        if not isinstance(data, IntervalData):
            # the reference's own prepare_data output: a list of IntervalItem (cluster.py:116-121)
            data = IntervalData.from_items(data)
        self.data = data
        self.csr = data.csr()
        self.ctx = ctx or Context(_default_device() if device is None else device)
        c = self.csr
        thr0 = np.where(c.iv_aln == 0, FSLR_THR_ZERO_ALN, 0).astype(np.int32)
        # reads of more than FSLR_MAX_L intervals: the library uploads them as FSLR_MAX_L-interval
        # chunks (fslr_set_reads_any); self.long = the real reads' lengths
        self.long = np.diff(np.asarray(c.read_off, np.int64)).astype(np.int32) if has_long_reads(c) else None
        if self.long is not None:
            self.ctx.load_csr_any(c, thr0)
        else:
            self.ctx.load_csr(c, thr0)
        self.ctx.build_index()


class RowsCSR:
    """The CSR fslr_set_reads_rows made on the device: the host holds what the CLI reads
    of it (the qname code of each read rank, the counts and flags); the columns are copied off the
    device on first use (fslr_get_csr) and then read as a ``prep.CSR``."""
    start_sorted = True

    def __init__(self, ctx, info):
        self._ctx, self._host = ctx, None
        self._n, self._ni = int(info['n_reads']), int(info['n_intervals'])
        self.n_chroms = int(info['n_chroms'])
        self.nal_varies = bool(info['nal_varies'])
        self.read_qcode = ctx.read_codes()

    n_reads = property(lambda self: self._n)
    n_intervals = property(lambda self: self._ni)

    def host(self) -> CSR:
        if self._host is None:
            d = self._ctx.device_csr(self._ni, self.n_chroms)
            self._host = CSR(read_off=d['read_off'], read_qlen2=d['read_qlen2'], read_nal=d['read_nal'],
                             iv_chrom=d['iv_chrom'], iv_start=d['iv_start'], iv_end=d['iv_end'], iv_aln=d['iv_aln'],
                             n_chroms=self.n_chroms, read_qcode=self.read_qcode, data_pos=d['data_pos'],
                             nal_varies=self.nal_varies, start_sorted=True)
        return self._host

    def __getattr__(self, name):                 # read_off, iv_*, data_pos: the host copy
        if name.startswith('_'):
            raise AttributeError(name)
        return getattr(self.host(), name)


class RowsIndex(DeviceIntervalIndex):
    """build_interval_trees' result for the columnar CLI: the reads set on the device from rows
    (fslr_set_reads_rows, thresholds folded there for ``overlap``) and the index built."""

    def __init__(self, data, csr: RowsCSR, ctx: Context, overlap: float):
        self.source = self.data = data
        self.csr, self.ctx, self.long = csr, ctx, None
        self.overlap = float(overlap)
        ctx.build_index()


class MultiGpuIndex:
    """What build_interval_trees returns for ``n_gpus > 1``: the prepared CSR on the host.  The ranks
    (one process per GPU, fslr_amd.multi) upload it and build their chromosomes' index inside
    query_interval_trees; this process must not have initialised the GPU before then."""

    def __init__(self, data, n_gpus: int, device: int | None = None):
        self.source = data
        if not isinstance(data, IntervalData):
            data = IntervalData.from_items(data)
        self.data = data
        self.csr = data.csr()
        self.n_gpus = int(n_gpus)
        self.first_device = 0 if device is None else int(device)


def _open_context(device: int | None = None) -> Context:
    """A library context on ``device`` (default $FSLR_DEVICE / $LOCAL_RANK / 0)."""
    return Context(_default_device() if device is None else int(device))


def build_interval_trees(data, device: int | None = None, n_gpus: int = 1, ctx: Context | None = None):
    """cluster.py:124-130: upload the prepared intervals and build the (chrom, start) index on the GPU.

    ``data`` is this module's ``prepare_data`` result or the reference's (a list of IntervalItem).
    ``n_gpus > 1``: the chromosome-split multi-GPU query; the upload happens in the
    per-GPU processes that query_interval_trees starts."""
    if int(n_gpus) > 1:
        return MultiGpuIndex(data, n_gpus, device)
    return DeviceIntervalIndex(data, device, ctx=ctx)


class ClusterGraph:
    """Graph of read pairs (the reference's ``nx.Graph``), held as device-computed labels.

    ``labels[r]`` = minimum rank in read r's connected component (ranks are the
    first-appearance order of reads in ``data``).  Nodes are the reads with at
    least one edge, as in ``G.add_edge`` (cluster.py:221).
    """

    def __init__(self, qnames_by_rank, labels, edges_ab, fwd, stats):
        self.qnames_by_rank = qnames_by_rank
        self.labels = labels
        self.edges_ab = edges_ab
        self.fwd = fwd
        self.stats = stats
        n = labels.shape[0]
        sizes = np.bincount(labels, minlength=n) if n else np.zeros(0, np.int64)
        self.comp_size = sizes[labels] if n else np.zeros(0, np.int64)
        self.node_mask = self.comp_size >= 2
        roots = np.flatnonzero((sizes >= 2))          # component roots = min ranks, ascending
        self.roots = roots
        cid = np.full(n, -1, dtype=np.int64)
        if n:
            rid = np.full(n, -1, dtype=np.int64)
            rid[roots] = np.arange(roots.size)
            cid = np.where(self.node_mask, rid[labels], -1)
        self.component_id = cid                        # per rank; -1 = not a node

    def number_of_nodes(self):
        return int(self.node_mask.sum())

    def number_of_edges(self):
        return int(self.edges_ab[0].shape[0])

    @property
    def nodes(self):
        return [self.qnames_by_rank[r] for r in np.flatnonzero(self.node_mask)]

    @property
    def edges(self):
        a, b = self.edges_ab
        return [(self.qnames_by_rank[x], self.qnames_by_rank[y]) for x, y in zip(a.tolist(), b.tolist())]

    def components(self):
        order = np.flatnonzero(self.node_mask)
        cid = self.component_id[order]
        srt = np.argsort(cid, kind='stable')
        out = [set() for _ in range(self.roots.size)]
        for c, r in zip(cid[srt].tolist(), order[srt].tolist()):
            out[c].add(self.qnames_by_rank[r])
        return out

    def to_networkx(self):
        import networkx as nx
        G = nx.Graph()
        G.add_edges_from(self.edges)
        return G


def query_interval_trees(interval_trees, data, overlap_cutoff, jaccard_threshold, edge_threshold, qlen_diff, diff):
    """cluster.py:187-227 on the GPU.

    Returns ``(match_df, G)``.  The pair kernels evaluate every candidate pair
    (E*); when a read has more than ``edge_threshold`` forward partners, the
    reference's per-read cap (cluster.py:223-224) is replayed exactly
    (``fslr_apply_edge_cap``; search order of the superintervals stand-in,
    SURVEY.md §8c).  ``match_df`` rows are the graph's edges as the reference
    records them — (read whose loop formed the edge, partner, I/U as a Python
    float) — sorted by (query1 rank, query2 rank); the reference's row order is
    set order (arbitrary).
    """
    g = query_graph(interval_trees, data, overlap_cutoff, jaccard_threshold, edge_threshold, qlen_diff, diff)
    return _graph_outputs(g.data.qnames[g.csr.read_qcode], g.labels, g.a, g.b, g.I, g.U, g.fwd, g.stats)


class RawGraph:
    """query_graph's result: the graph over read ranks without qname strings (the CLI's columnar
    path maps ranks to qname codes itself).  Edges sorted by (a, b).

    ``a, b, I, U`` and ``fwd`` are arrays, or — from a single-GPU query — ``edges`` / ``fwd`` loaders
    that copy them off the device on first use (the CLI needs only the labels and the edge count)."""

    def __init__(self, data, csr, labels, a=None, b=None, I=None, U=None, fwd=None, st=None, *, edges=None,
                 n_edges=None):
        self.data, self.csr, self.labels, self.stats = data, csr, labels, st
        self._raw = (a, b, I, U) if edges is None else edges
        self._fwd = fwd
        self._sorted = None
        self.n_edges = int(a.shape[0]) if n_edges is None else int(n_edges)

    @property
    def fwd(self):
        if callable(self._fwd):
            self._fwd = self._fwd()
        return self._fwd

    def _edges(self):
        if self._sorted is None:                    # fetched and sorted on first use
            raw = self._raw() if callable(self._raw) else self._raw
            a, b, I, U = raw
            order = np.lexsort((b, a))
            self._sorted = (a[order], b[order], I[order], U[order])
            self._raw = None
        return self._sorted

    a = property(lambda self: self._edges()[0])
    b = property(lambda self: self._edges()[1])
    I = property(lambda self: self._edges()[2])
    U = property(lambda self: self._edges()[3])


def query_graph(interval_trees, data, overlap_cutoff, jaccard_threshold, edge_threshold, qlen_diff, diff):
    """query_interval_trees without the match_df / qname outputs: a RawGraph."""
    min(jaccard_threshold)                              # cluster.py:188 raises on an empty list
    if isinstance(interval_trees, MultiGpuIndex) and (interval_trees.source is data or interval_trees.data is data):
        mg = interval_trees
        thr = fold_overlap_threshold(mg.csr.iv_aln, overlap_cutoff)
        # the sweep split, or for overlap <= 0, an aln_size == 0 interval or reads of more than 64
        # intervals the query-shard split
        return _query_multi_gpu(mg, thr, jaccard_threshold, edge_threshold, qlen_diff, diff)
    if not isinstance(interval_trees, DeviceIntervalIndex) or (interval_trees.source is not data and
                                                               interval_trees.data is not data):
        interval_trees = DeviceIntervalIndex(data)
    idx = interval_trees
    data = idx.data
    csr = idx.csr
    ctx = idx.ctx
    if csr.nal_varies:
        warnings.warn('n_alignments differs between rows of one read; the reference then uses the row its '
                      'search reaches first (order-dependent); the first row in data order is used', EdgeCapWarning)
    if idx.long is not None:
        return _query_long(idx, overlap_cutoff, jaccard_threshold, edge_threshold, qlen_diff, diff)
    if isinstance(idx, RowsIndex):
        if idx.overlap != float(overlap_cutoff):             # folded on the device at the upload
            ctx.fold_thresholds(overlap_cutoff)
            idx.overlap = float(overlap_cutoff)
    else:
        ctx.set_thresholds(fold_overlap_threshold(csr.iv_aln, overlap_cutoff))
    pt = pass_table(jaccard_threshold)
    qcut = 1 - qlen_diff
    ncut = 1 - diff
    ctx.reserve_edges(max(1 << 16, 12 * csr.n_reads))
    st = ctx.run_query(qcut, ncut, pt, int(edge_threshold))
    st['cap'] = ctx.apply_edge_cap(int(edge_threshold))
    st['n_edges'] = ctx.stats()['n_edges']
    st['max_fwd'] = st['cap']['max_fwd']
    ctx.components()
    labels = ctx.labels()
    ne = st['n_edges']
    # the edges and forward degrees stay in HBM until asked for (query_interval_trees does at once;
    # the CLI never does); this context's next query would replace them
    gen = ctx.query_gen = getattr(ctx, 'query_gen', 0) + 1

    def fetch(what):
        if getattr(ctx, 'query_gen', 0) != gen:
            raise RuntimeError('the graph\'s context has run another query since')
        return ctx.edges(ne) if what == 'edges' else ctx.fwd_degree()
    return RawGraph(data, csr, labels, fwd=lambda: fetch('fwd'), st=st, edges=lambda: fetch('edges'), n_edges=ne)


def _graph_outputs(qnames_by_rank, labels, a, b, I, U, fwd, st):
    order = np.lexsort((b, a))
    a, b, I, U = a[order], b[order], I[order], U[order]
    ne = int(a.shape[0])
    match_df = pd.DataFrame({'query1': qnames_by_rank[a] if ne else np.zeros(0, object),
                             'query2': qnames_by_rank[b] if ne else np.zeros(0, object),
                             'jaccard_similarity': I / U if ne else np.zeros(0)})
    return match_df, ClusterGraph(qnames_by_rank, labels, (a, b), fwd, st)


def _query_long(idx, overlap_cutoff, jaccard_threshold, edge_threshold, qlen_diff, diff):
    """query_interval_trees with reads of more than FSLR_MAX_L intervals.

    E*: where the sweep's gates apply (overlap > 0, no aln_size == 0 interval, no long read with qlen2
    or n_alignments 0), the sweep over the virtual CSR writes every match entry; pairs of two short
    reads are decided by its pair stage, pairs with a long read by the first-fit over their whole
    lists (fslr_long_query).  Otherwise every distinct pair goes through the general evaluator
    (fslr_long_pairs).  When a read has more than ``edge_threshold`` forward edges, the reference's
    per-read cap (cluster.py:223-224) is replayed over E* in the real-read space
    (fslr_cap_replay_pairs)."""
    csr, ctx = idx.csr, idx.ctx
    rlen = idx.long
    n = csr.n_reads
    thr = fold_overlap_threshold(csr.iv_aln, overlap_cutoff)           # the real CSR's order
    lg = rlen > FSLR_MAX_L
    fast = (multi.sweep_applies(csr, thr) and not (csr.read_qlen2[lg] == 0).any()
            and not (csr.read_nal[lg] == 0).any())
    ctx.set_thresholds(thr)
    ctx.set_long_cutoffs(umax_table(jaccard_threshold, int(rlen.max())))
    pt = pass_table(jaccard_threshold)
    qcut, ncut = 1 - qlen_diff, 1 - diff
    ctx.reserve_edges(max(1 << 16, 12 * n))
    if fast:
        while True:
            n_long = ctx.long_query(qcut, ncut, pt, int(edge_threshold))
            st = ctx.stats(check=False)
            if st['n_edges'] <= st['edge_capacity']:
                break
            ctx.reserve_edges(int(st['n_edges'] * 1.25) + 4096)
        st = ctx.stats()
        la, lb, lI, lU = ctx.long_edges(n_long)
        a, b, I, U = ctx.edges(st['n_edges'])
        a, b = np.concatenate([a, la]), np.concatenate([b, lb])
        I, U = np.concatenate([I, lI]), np.concatenate([U, lU])
        engine = 'sweep+long'
    else:
        n_long = ctx.long_pairs(qcut, ncut, pt, int(edge_threshold))
        st = ctx.stats()
        a, b, I, U = ctx.long_edges(n_long)
        engine = 'pairs'
    fwd = np.bincount(a, minlength=n).astype(np.int32)
    max_fwd = int(fwd.max()) if n else 0
    if st.get('zd_pairs', 0) and max_fwd <= int(edge_threshold):
        # every loop runs to its end, so each listed pair is visited (cluster.py:178-183, 133-136); with
        # the cap binding the replay decides (fslr_cap_replay_pairs raises where a loop reaches one)
        raise ZeroDivisionError('division by zero')
    cap = {'applied': 0, 'max_fwd': max_fwd}
    if max_fwd > int(edge_threshold):
        # the capped graph: edge k kept when formed in a loop, re-oriented as (former, partner)
        who, fwd, cap = ctx.cap_replay_pairs(int(edge_threshold), a, b, n)
        keep = who != 2
        a, b = np.where(who == 0, a, b)[keep], np.where(who == 0, b, a)[keep]
        I, U = I[keep], U[keep]
        ctx.components()
        labels = ctx.labels()[:n]
    elif fast:
        ctx.components()
        if n_long:
            ctx.union_pairs(la, lb, n_long, on_device=False)
            ctx.finalize_labels()
        labels = ctx.labels()[:n]
    else:
        ctx.components()
        labels = ctx.labels()[:n]
    st = dict(st, engine=engine, n_edges=int(a.shape[0]), max_fwd=max_fwd, long_reads=int(lg.sum()),
              long_pair_edges=int(n_long), cap=cap)
    return RawGraph(idx.data, csr, labels, a, b, I, U, fwd, st)


def _query_multi_gpu(mg, thr, jaccard_threshold, edge_threshold, qlen_diff, diff):
    """query_interval_trees over ``mg.n_gpus`` ranks (fslr_amd.multi): same edges, forward degrees and
    labels as one GPU (union of per-chromosome matchings, label union; the cap replayed on rank 0)."""
    data, csr = mg.data, mg.csr
    if csr.nal_varies:
        warnings.warn('n_alignments differs between rows of one read; the reference then uses the row its '
                      'search reaches first (order-dependent); the first row in data order is used', EdgeCapWarning)
    r = multi.query(csr, thr, 1 - qlen_diff, 1 - diff, pass_table(jaccard_threshold), int(edge_threshold),
                    mg.n_gpus, first_device=mg.first_device, cutoffs=list(jaccard_threshold))
    a, b, I, U = r['edges']
    st = {'engine': r.get('path', 'sweep'), 'n_gpus': mg.n_gpus, 'backend': r['backend'], 'evaluated_pairs': -1,
          'n_edges': int(a.shape[0]), 'max_fwd': r['max_fwd'], 'cap': r['cap'], 'capped': r['capped']}
    return RawGraph(data, csr, np.asarray(r['labels']), a, b, I, U, r['fwd'], st)


def get_subgraphs(G):
    """cluster.py:230-234: connected components, in the reference's order (by min read rank)."""
    if isinstance(G, ClusterGraph):
        return G.components()
    import networkx as nx
    return list(nx.connected_components(G))


def choose_alignment(bed_file):
    """cluster.py:237-254: per cluster the read with the highest mean alignment_score (first on ties)."""
    fast = _choose_alignment_codes(bed_file)
    if fast is not None:
        return fast
    avg = bed_file.groupby('qname')['alignment_score'].mean()
    bed_file['avg_alignment_score'] = bed_file['qname'].map(avg)
    sel = bed_file.groupby('cluster')['avg_alignment_score'].idxmax()
    chosen = bed_file.loc[sel.to_numpy(), 'qname']
    return bed_file[bed_file['qname'].isin(chosen)]


def _choose_alignment_codes(bed_file):
    """choose_alignment from the reader's qname codes (ingest.QnameCodes), for an int64
    alignment_score and numeric cluster ids, or None.

    groupby('qname').mean() of int64 scores: the float64 sum of integers below 2**53 is exact in any
    order (pandas' compensated sum included), divided by the count, so bincount gives the same
    doubles.  groupby('cluster').idxmax() = the first row (in frame order) holding its cluster's
    maximum; scores and clusters are constant per qname, so it is the earliest first row among
    the cluster's qnames with the maximal mean."""
    if not isinstance(bed_file.attrs.get(ingest.ATTR), ingest.QnameCodes) or 'cluster' not in bed_file:
        return None
    score = bed_file['alignment_score'].to_numpy()
    cl = bed_file['cluster'].to_numpy()
    if score.dtype != np.int64 or cl.dtype.kind not in 'iuf' or not len(cl):
        return None
    if np.abs(score).max() >= (1 << 53) // max(1, len(score)):
        return None
    codes, uniq = ingest.factorize_qname(bed_file)
    nq = len(uniq)
    sums = np.bincount(codes, weights=score.astype(np.float64), minlength=nq)
    cnt = np.bincount(codes, minlength=nq)
    avg_q = sums / cnt
    with warnings.catch_warnings():
        warnings.simplefilter('ignore')
        bed_file['avg_alignment_score'] = avg_q[codes]
    first_row = np.full(nq, -1, dtype=np.int64)
    first_row[codes[::-1]] = np.arange(len(codes) - 1, -1, -1)
    cl_q = cl[first_row]
    if cl.dtype.kind == 'f':
        if np.isnan(cl_q).any() or (cl_q != np.floor(cl_q)).any() or cl_q.min() < 0:
            return None
    if (cl != cl_q[codes]).any():                      # cluster not constant per qname
        return None
    cid = cl_q.astype(np.int64)
    k = int(cid.max()) + 1
    best = np.full(k, -np.inf)
    np.maximum.at(best, cid, avg_q)
    cand = np.flatnonzero(avg_q == best[cid])
    win_row = np.full(k, len(codes), dtype=np.int64)
    np.minimum.at(win_row, cid[cand], first_row[cand])
    chosen = np.zeros(nq, dtype=bool)
    chosen[codes[win_row[win_row < len(codes)]]] = True
    return bed_file[chosen[codes]]
