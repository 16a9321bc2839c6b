"""Synthetic ``.mappings.bed`` generator.

The reference ships no data, so every parity fixture and every bench input is
synthesised here.  The generator writes the column layout produced by the
reference's BAM→BED step (``collect_mapping_info.py:176-177``) with rows in its
order ``(n_alignments desc, qname asc, qstart asc)`` (``collect_mapping_info.py:174``).

Model (seeded numpy PCG64, one draw order per seed):

* 23 chromosomes ``chr1..chr22, chrX`` of 150 Mb each (the BAM-header stand-in).
* "Events" of ``min(cluster_cap, Geometric(1/3))`` reads each.  An event has
  ``L`` fillings, ``U{1..lmax}`` (``dist='uniform'``) or a truncated Zipf(1.5)
  on ``1..lmax`` (``dist='zipf'``, config 5).
* A filling sits on a uniform chromosome, start ``U[1 Mb, 140 Mb)`` (outside the
  subtelomere mask), length ``U[300, 5000]``.  Each read of the event jitters
  start and length by ±20 bp; starts are re-drawn until every filling start is
  globally distinct (no ``sort_values('start')`` tie hazard).
* Rows per read: a 20 bp "bread" at qstart 0, the fillings in query order
  (qstart cumulative from 20), a 20 bp bread at the end.  ``n_alignments = L+2``,
  ``aln_size = length``, ``alignment_score = length``.

``SynthBed`` keeps everything columnar; ``qname`` strings are only built when a
DataFrame / TSV is requested, so the 1M / 10M read bench inputs stay cheap.
"""
from __future__ import annotations

import dataclasses

import numpy as np

CHROMS = [f"chr{i}" for i in range(1, 23)] + ["chrX"]
CHROM_LEN = 150_000_000
BED_COLUMNS = ['chrom', 'rstart', 'rend', 'qname', 'n_alignments', 'aln_size', 'qstart', 'qend',
               'strand', 'mapq', 'qlen', 'alignment_score', 'short_anchor<50bp', 'fslr_version',
               'inferred_by_primer', 'seq']


@dataclasses.dataclass
class SynthBed:
    """Columnar ``.mappings.bed`` rows in file order."""
    chrom_names: list            # index → chromosome name
    chrom: np.ndarray            # int32 index into chrom_names
    rstart: np.ndarray           # int64
    rend: np.ndarray             # int64
    read_id: np.ndarray          # int64 row → read number (qname = name_of(read_id))
    n_alignments: np.ndarray     # int64
    aln_size: np.ndarray         # int64
    qstart: np.ndarray           # int64
    qend: np.ndarray             # int64
    qlen: np.ndarray             # int64
    alignment_score: np.ndarray  # int64
    chrom_lengths: dict          # header: name → length
    n_reads: int
    name_prefix: str = "read"
    name_suffix: str = ".21q1F_17p6R"

    @property
    def n_rows(self) -> int:
        return int(self.chrom.shape[0])

    def qnames(self) -> np.ndarray:
        """Row qnames as an object array (built on demand)."""
        names = np.array([f"{self.name_prefix}{i:08d}{self.name_suffix}" for i in range(self.n_reads)],
                         dtype=object)
        return names[self.read_id]

    def to_dataframe(self):
        import pandas as pd
        n = self.n_rows
        chrom = np.asarray(self.chrom_names, dtype=object)[self.chrom]
        first_row = np.ones(n, dtype=bool)
        first_row[1:] = self.read_id[1:] != self.read_id[:-1]
        seq = np.where(first_row, 'ACGTACGTAC', '')
        short_anchor = np.ones(n, dtype=np.int64)    # breads are 20 bp < 50 bp (collect_mapping_info.py:166-172)
        df = pd.DataFrame({
            'chrom': chrom,
            'rstart': self.rstart,
            'rend': self.rend,
            'qname': self.qnames(),
            'n_alignments': self.n_alignments,
            'aln_size': self.aln_size,
            'qstart': self.qstart,
            'qend': self.qend,
            'strand': np.full(n, '+', dtype=object),
            'mapq': np.full(n, 60, dtype=np.int64),
            'qlen': self.qlen,
            'alignment_score': self.alignment_score,
            'short_anchor<50bp': short_anchor,
            'fslr_version': np.full(n, '0.3.10', dtype=object),
            'inferred_by_primer': np.zeros(n, dtype=np.int64),
            'seq': seq,
        })
        return df[BED_COLUMNS]

    def write_tsv(self, path: str) -> None:
        """``to_dataframe().to_csv(path, sep='\\t', index=False)``; the same bytes through pyarrow's
        threaded CSV writer when it is importable (10M reads: minutes with pandas)."""
        df = self.to_dataframe()
        try:
            import pyarrow as pa
            import pyarrow.csv as pcsv
        except ImportError:                      # pragma: no cover - pyarrow ships in this image
            df.to_csv(path, sep='\t', index=False)
            return
        with open(path, 'wb') as fh:
            fh.write(('\t'.join(df.columns) + '\n').encode())
            pcsv.write_csv(pa.Table.from_pandas(df, preserve_index=False), fh,
                           pcsv.WriteOptions(include_header=False, delimiter='\t', quoting_style='none'))

    def interval_data(self, cluster_mask=('subtelomere',), threshold: int = 500_000):
        """The prepared ``data`` (fslr_amd.prep.IntervalData) straight from the columns.

        Same host stages as the DataFrame path (rename → keep_fillings →
        prepare_data → mask, main.py:227-237) on numeric columns; qname strings
        are materialised lazily (``LazyNames``).  Checked against the DataFrame
        path by tests/test_synth.py.
        """
        from .prep import IntervalData, data_order, first_last_masks, group_span, mask_keep
        first, last = first_last_masks(self.read_id)
        keep = ~(first | last)
        qlen2 = group_span(self.read_id[keep], self.qstart[keep], self.qend[keep], self.n_reads)
        rid = self.read_id[keep]
        rs, re_ = self.rstart[keep], self.rend[keep]
        start = np.minimum(rs, re_)
        end = np.maximum(rs, re_)
        aln = self.aln_size[keep]
        # rename_chromosomes numbering: chrN by N (all synthetic names are chrN / chrX)
        names = self.chrom_names
        key = [(0, int(n[3:])) if n[3:].isdigit() else (1, i) for i, n in enumerate(names)]
        order_names = sorted(range(len(names)), key=lambda i: key[i])
        num = np.empty(len(names), dtype=np.int64)
        num[order_names] = np.arange(1, len(names) + 1)
        chrom = num[self.chrom[keep]]
        order = data_order(start)
        lens = {int(num[names.index(k)]): v for k, v in self.chrom_lengths.items() if k in names}
        mask = [m if m == 'subtelomere' else int(num[names.index(m)]) for m in cluster_mask if
                m == 'subtelomere' or m in names]
        data = IntervalData(chrom=chrom[order], start=start[order].astype(np.int64), end=end[order].astype(np.int64),
                            aln_size=aln[order].astype(np.int64), qcode=rid[order].astype(np.int64),
                            qnames=LazyNames(self.name_prefix, self.name_suffix, self.n_reads),
                            n_alignments=self.n_alignments[keep][order].astype(np.int64),
                            qlen2=qlen2[rid][order].astype(np.int64),
                            middle=(aln // 2 + start)[order].astype(np.int64),
                            index=np.flatnonzero(keep)[order])
        if mask:
            data = data.select(mask_keep(data.chrom, data.start, data.end, mask, lens, threshold))
        return data


class LazyNames:
    """code → qname, formatted on access (indexable like the object array of the DataFrame path)."""

    def __init__(self, prefix, suffix, n):
        self.prefix, self.suffix, self.n = prefix, suffix, n

    def __len__(self):
        return self.n

    def _one(self, i):
        return f"{self.prefix}{int(i):08d}{self.suffix}"

    def __getitem__(self, k):
        if isinstance(k, (int, np.integer)):
            return self._one(k)
        return np.array([self._one(i) for i in np.asarray(k).ravel()], dtype=object).reshape(np.shape(k))


def _zipf_trunc(rng, a: float, lmax: int, size: int) -> np.ndarray:
    k = np.arange(1, lmax + 1, dtype=np.float64)
    pmf = k ** (-a)
    cdf = np.cumsum(pmf / pmf.sum())
    u = rng.random(size)
    return (np.searchsorted(cdf, u, side='right') + 1).clip(1, lmax).astype(np.int64)


def _member(sorted_arr: np.ndarray, x: np.ndarray) -> np.ndarray:
    if sorted_arr.size == 0:
        return np.zeros(x.shape, dtype=bool)
    pos = np.minimum(np.searchsorted(sorted_arr, x), sorted_arr.size - 1)
    return sorted_arr[pos] == x


def generate(n_reads: int, lmax: int, seed: int, dist: str = 'uniform', cluster_cap: int = 10,
             lmin: int = 1, size_p: float = 1.0 / 3.0, chrom_weights=None) -> SynthBed:
    """Generate ``n_reads`` reads (SURVEY §8d model).  Deterministic in ``seed``.

    ``cluster_cap``/``size_p`` set the event size ``min(cluster_cap, Geometric(size_p))``;
    the default keeps every read's forward degree <= 9 (edge cap never binds).
    """
    rng = np.random.Generator(np.random.PCG64(seed))
    # events and their sizes
    sizes = np.minimum(cluster_cap, rng.geometric(size_p, size=max(n_reads, 1))).astype(np.int64)
    cs = np.cumsum(sizes)
    n_ev = int(np.searchsorted(cs, n_reads) + 1) if n_reads > 0 else 0
    sizes = sizes[:n_ev].copy()
    if n_ev:
        sizes[-1] -= int(cs[n_ev - 1] - n_reads)
    if dist == 'uniform':
        ev_L = rng.integers(lmin, lmax + 1, size=n_ev).astype(np.int64)
    elif dist == 'zipf':
        ev_L = np.maximum(_zipf_trunc(rng, 1.5, lmax, n_ev), lmin)
    else:
        raise ValueError(dist)
    ev_off = np.zeros(n_ev + 1, dtype=np.int64)
    np.cumsum(ev_L, out=ev_off[1:])
    n_ev_fill = int(ev_off[-1])
    if chrom_weights is None:
        ev_chrom = rng.integers(0, len(CHROMS), size=n_ev_fill).astype(np.int32)
    else:                                        # a skewed genome (e.g. a targeted panel): chromosome weights
        w = np.asarray(chrom_weights, np.float64)
        ev_chrom = rng.choice(len(CHROMS), size=n_ev_fill, p=w / w.sum()).astype(np.int32)
    ev_start = rng.integers(1_000_000, 140_000_000, size=n_ev_fill).astype(np.int64)
    ev_len = rng.integers(300, 5001, size=n_ev_fill).astype(np.int64)

    # reads → events; fillings per read
    read_ev = np.repeat(np.arange(n_ev, dtype=np.int64), sizes)
    read_L = ev_L[read_ev]
    read_off = np.zeros(n_reads + 1, dtype=np.int64)
    np.cumsum(read_L, out=read_off[1:])
    nf = int(read_off[-1])
    f_read = np.repeat(np.arange(n_reads, dtype=np.int64), read_L)
    f_local = np.arange(nf, dtype=np.int64) - read_off[f_read]
    f_ev_fill = ev_off[read_ev[f_read]] + f_local
    f_chrom = ev_chrom[f_ev_fill]
    f_start = ev_start[f_ev_fill] + rng.integers(-20, 21, size=nf)
    f_len = ev_len[f_ev_fill] + rng.integers(-20, 21, size=nf)

    # globally distinct starts: keep the first (stable order) of every value, re-draw
    # the jitter of the others until they hit a free value (membership in a bitmap of used
    # values; same draws and outcome as a sorted-set test)
    order = np.argsort(f_start, kind='stable')
    s_sorted = f_start[order]
    dup_sorted = np.zeros(nf, dtype=bool)
    if nf > 1:
        dup_sorted[1:] = s_sorted[1:] == s_sorted[:-1]
    pending = np.sort(order[dup_sorted])
    del order, s_sorted, dup_sorted
    lo_v = int(ev_start.min()) - 6000 if ev_start.size else 0
    hi_v = int(ev_start.max()) + 6000 if ev_start.size else 1
    used = np.zeros(hi_v - lo_v, dtype=bool)
    used[f_start - lo_v] = True
    jit = 20
    for it in range(400):
        if pending.size == 0:
            break
        if it >= 8:
            jit = min(jit * 2, 5000)
        cand = ev_start[f_ev_fill[pending]] + rng.integers(-jit, jit + 1, size=pending.size)
        clash = used[cand - lo_v]
        _, first = np.unique(cand, return_index=True)
        firstmask = np.zeros(pending.size, dtype=bool)
        firstmask[first] = True
        ok = ~clash & firstmask
        f_start[pending[ok]] = cand[ok]
        used[cand[ok] - lo_v] = True
        pending = pending[~ok]
    else:  # pragma: no cover
        raise RuntimeError("could not make filling starts distinct")
    del used

    # query coordinates: fillings start at qstart 20, contiguous
    csum = np.cumsum(f_len)
    read_len_sum = np.zeros(n_reads, dtype=np.int64)
    np.add.at(read_len_sum, f_read, f_len)
    before = csum - f_len - np.concatenate([[0], csum])[read_off[f_read]]
    f_qstart = 20 + before
    f_qend = f_qstart + f_len

    # read order in the file: (n_alignments desc, qname asc); qname = read number,
    # numbered by a random permutation so that event mates are not adjacent
    read_name = rng.permutation(n_reads).astype(np.int64)
    read_order = np.lexsort((read_name, -(read_L + 2)))

    # assemble rows: bread, fillings..., bread per read (in read_order)
    rows_per = read_L + 2
    out_L = rows_per[read_order]
    out_off = np.zeros(n_reads + 1, dtype=np.int64)
    np.cumsum(out_L, out=out_off[1:])
    n_rows = int(out_off[-1])
    pos_of_read = np.empty(n_reads, dtype=np.int64)
    pos_of_read[read_order] = np.arange(n_reads, dtype=np.int64)
    base = out_off[pos_of_read]            # first row of each read
    row_read = np.repeat(read_order, out_L)

    chrom_names = list(CHROMS)
    chrom = np.empty(n_rows, dtype=np.int32)
    rstart = np.empty(n_rows, dtype=np.int64)
    rend = np.empty(n_rows, dtype=np.int64)
    aln = np.empty(n_rows, dtype=np.int64)
    qs = np.empty(n_rows, dtype=np.int64)
    qe = np.empty(n_rows, dtype=np.int64)

    fr = base[f_read] + 1 + f_local
    chrom[fr] = f_chrom
    rstart[fr] = f_start
    rend[fr] = f_start + f_len
    aln[fr] = f_len
    qs[fr] = f_qstart
    qe[fr] = f_qend

    b1 = base
    b2 = base + read_L + 1
    chrom[b1] = chrom_names.index('chr21')
    chrom[b2] = chrom_names.index('chr17')
    rstart[b1] = CHROM_LEN - 10_000
    rend[b1] = CHROM_LEN - 10_000 + 20
    rstart[b2] = CHROM_LEN - 20_000
    rend[b2] = CHROM_LEN - 20_000 + 20
    aln[b1] = 20
    aln[b2] = 20
    qs[b1] = 0
    qe[b1] = 20
    qs[b2] = 20 + read_len_sum
    qe[b2] = 40 + read_len_sum

    qlen_read = read_len_sum + 200
    return SynthBed(
        chrom_names=chrom_names, chrom=chrom, rstart=rstart, rend=rend,
        read_id=read_name[row_read], n_alignments=(read_L + 2)[row_read],
        aln_size=aln, qstart=qs, qend=qe, qlen=qlen_read[row_read], alignment_score=aln.copy(),
        chrom_lengths={c: CHROM_LEN for c in chrom_names}, n_reads=n_reads)
