"""``{name}.bwa_dodi.bam`` → ``{name}.mappings.bed``: the producer of the clustering input
(reference ``fslr/collect_mapping_info.py:19-181``).

Same entry point and output as the reference's ``mapping_info(f, outf, regions_path, primers)``.
The records come from the native decoder (:class:`fslr_amd.bam.BamFile`) as columns instead of
pysam objects; the per-read logic is vectorised over them, and the two sorts and the writer are
the reference's own pandas calls on a frame with the same rows, row order and dtypes, so ties
and number formatting are the reference's.

Reference → here:
  get_query_pos_from_cigartuples  :7-17     clip_first / read_len - clip_last / read_len columns
  group by qname (defaultdict)    :22-26    first-appearance codes of the mapped records
  primary choice                  :38-47    first record without flag & 2304; several: first max AS
  strand flip vs the primary      :56-62
  rows                            :74-105   columnar
  'missing bread' primer rows     :114-163  single-record reads only (few), per read
  sorts + short-anchor flag       :167-181  the same pandas calls
"""
from __future__ import annotations

import numpy as np
import pandas as pd

from .bam import BamFile

REFERENCE_VERSION = '0.3.10'      # version("fslr") of the reference this reproduces (setup.py:6)

OUT_COLUMNS = ['chrom', 'rstart', 'rend', 'qname', 'n_alignments', 'aln_size', 'qstart', 'qend', 'strand', 'mapq',
               'qlen', 'alignment_score', 'short_anchor<50bp', 'fslr_version', 'inferred_by_primer', 'seq']


def get_query_pos_from_cigartuples(read_len, clip_first, clip_last):
    """collect_mapping_info.py:7-17 over columns: (start, end, query_length) on the read as
    sequenced, hard clips included."""
    return clip_first, read_len - clip_last, read_len


def _read_regions(regions_path):
    regions = {}
    if regions_path:
        with open(regions_path) as fh:                 # :31-37
            for line in fh:
                f = line.strip().split('\t')
                regions.setdefault(f[0], []).append((int(f[1]), int(f[2])))
    return regions


def mapping_info(f, outf, regions_path, primers, n_threads: int = 0, version: str = REFERENCE_VERSION):
    """collect_mapping_info.py:19-181."""
    with BamFile(f, n_threads) as bam:
        return _mapping_info(bam, f, outf, regions_path, primers, version)


def _fail(*msg):
    print(*msg)
    raise SystemExit(None)                             # the reference's quit()


def _mapping_info(bam, f, outf, regions_path, primers, version):
    c = bam.columns
    mapped = np.flatnonzero((c['flag'] & 4) == 0)      # :24-26
    flag = c['flag'][mapped]
    qn = bam.qname[mapped]
    codes, uniq = pd.factorize(qn, sort=False)         # defaultdict insertion order
    n_rec, n_grp = len(mapped), len(uniq)
    # records grouped by read (file order inside a read)
    order = np.argsort(codes, kind='stable')
    gstart = np.searchsorted(codes[order], np.arange(n_grp + 1))
    size = np.diff(gstart)
    as_kind = c['as_kind'][mapped]
    as_tag = c['as_tag'][mapped]

    # primary per read (:38-47): records without flag & 2304; several -> the first with max AS
    cand = (flag & 2304) == 0
    n_cand = np.bincount(codes[cand], minlength=n_grp)
    err_rank = np.full(n_grp, 99, dtype=np.int64)       # the first failing read in order wins
    multi = n_cand > 1
    if multi.any():
        bad_as = np.zeros(n_grp, dtype=bool)
        sel = cand & multi[codes]
        np.logical_or.at(bad_as, codes[sel & (as_kind != 1)], True)
        err_rank[bad_as] = 0                           # get_tag('AS') KeyError in max()
    err_rank[(n_cand != 1) & ~multi & (err_rank > 1)] = 1
    pri_pos = np.full(n_grp, -1, dtype=np.int64)       # each read's primary record (mapped numbering)
    oc = order[cand[order]]                            # candidates, grouped, file order inside
    if oc.size:
        g = codes[oc]
        key_as = np.where(as_kind[oc] == 1, as_tag[oc], 0)     # reads lacking AS here raised above
        # first max AS per read: sort by (read, -AS, file position), take the first of each read
        srt = np.lexsort((oc, -key_as, g)) if multi.any() else np.arange(oc.size)
        first = np.ones(oc.size, dtype=bool)
        first[1:] = g[srt][1:] != g[srt][:-1]
        pri_pos[g[srt][first]] = oc[srt][first]
    no_as = np.zeros(n_grp, dtype=bool)
    np.logical_or.at(no_as, codes[as_kind != 1], True)
    err_rank[no_as & (err_rank > 2)] = 2               # get_tag('AS') KeyError building the rows
    pri_rec = np.where(pri_pos >= 0, pri_pos, 0)
    l_seq = c['l_seq'][mapped]
    no_seq = (pri_pos >= 0) & (l_seq[pri_rec] == 0)
    err_rank[no_seq & (err_rank > 3)] = 3              # 'missing' (:108-110)
    bad = np.flatnonzero(err_rank < 99)
    if bad.size:
        gb = int(bad[0])
        kind = int(err_rank[gb])
        recs = order[gstart[gb]:gstart[gb + 1]]
        if kind == 0 or kind == 2:
            raise KeyError("tag 'AS' not present")
        if kind == 1:
            _fail('Error in ', f, 'flag problem', int(n_cand[gb]), [int(x) for x in flag[recs]])
        _fail('missing', uniq[gb], [int(c['read_len'][mapped][r]) for r in recs])

    # per-record fields (:50-105)
    rev = (flag & 16) != 0
    pri_rev = rev[pri_rec][codes]
    qstart, qend, qlen = get_query_pos_from_cigartuples(c['read_len'][mapped], c['clip_first'][mapped],
                                                        c['clip_last'][mapped])
    flip = rev != pri_rev
    st = np.where(flip, qlen - qend, qstart)
    qend = np.where(flip, st + qend - qstart, qend)
    qstart = st
    tid = c['tid'][mapped]
    names = np.asarray(bam.references + [''], dtype=object)
    chrom = names[np.where((tid >= 0) & (tid < len(bam.references)), tid, len(bam.references))]
    rstart = c['pos'][mapped] + 1
    rend = c['pos'][mapped] + c['ref_span'][mapped]
    seq = np.full(n_rec, '', dtype=object)
    for r in pri_pos.tolist():
        seq[r] = bam.forward_sequence(int(mapped[r]))
    regions = _read_regions(regions_path)
    overlaps = np.zeros(n_rec, dtype=np.int64)
    for ch, ivs in regions.items():
        on = chrom == ch
        if not on.any():
            continue
        hit = np.zeros(int(on.sum()), dtype=bool)
        a, b = rstart[on], rend[on]
        for lo, hi in ivs:                             # pd.Interval(a, b].overlaps((lo, hi]): a < hi, lo < b
            hit |= (a < hi) & (lo < b)
        overlaps[on] = hit
    n_al = size[codes]
    frame = pd.DataFrame({'qname': qn, 'n_alignments': n_al, 'chrom': chrom, 'rstart': rstart, 'rend': rend,
                          'strand': np.where(rev, '-', '+').astype(object), 'qstart': qstart, 'qend': qend,
                          'qlen': qlen, 'aln_size': qend - qstart, 'mapq': c['mapq'][mapped].astype(np.int64),
                          'alignment_score': as_tag, 'seq': seq, 'fslr_version': version,
                          'inferred_by_primer': np.zeros(n_rec, dtype=np.int64)})
    if regions:
        frame['overlaps_region'] = overlaps
    frame = frame.iloc[order].reset_index(drop=True)   # reads in first-appearance order (res += temp)

    # 'missing bread' (:112-163): one-record reads with a gap <= 5 at an end get a primer row
    rows_before, rows_after = {}, {}
    singles = np.flatnonzero(size == 1)
    for g in singles.tolist():
        i = int(gstart[g])
        row = frame.iloc[i]
        qs, qe, ql = int(row['qstart']), int(row['qend']), int(row['qlen'])
        p_names = row['qname'].split('.')[-1].split('_')
        p1, p2 = [x.rstrip('FR') for x in p_names]
        if qs > 5 and ql - qe > 5:
            continue
        base = {'qname': row['qname'], 'n_alignments': 2, 'rstart': 0, 'rend': 0, 'qlen': ql, 'aln_size': 0,
                'mapq': 0, 'alignment_score': 0, 'seq': '', 'fslr_version': version, 'inferred_by_primer': 1}
        if p1 != 'False':
            rows_before[i] = dict(base, chrom=p1, strand='-' if p_names[0][-1] == 'R' else '+', qstart=0,
                                  qend=len(primers[p1]))
        elif p2 != 'False':
            rows_after[i] = dict(base, chrom=p2, strand='-' if p_names[1][-1] == 'R' else '+',
                                 qstart=ql - len(primers[p2]), qend=ql)
    if rows_before or rows_after:
        touched = np.array(sorted(set(rows_before) | set(rows_after)), dtype=np.int64)
        frame.loc[touched, 'n_alignments'] = 2
        extra = pd.DataFrame([rows_before.get(i) or rows_after.get(i) for i in touched.tolist()])
        # position keys: the primer row sorts just before (p1) or after (p2) its read's row
        key = np.concatenate([np.arange(len(frame), dtype=np.float64),
                              touched + np.array([-0.5 if i in rows_before else 0.5 for i in touched.tolist()])])
        frame = pd.concat([frame, extra[[c for c in frame.columns if c in extra.columns]]], ignore_index=True)
        frame = frame.iloc[np.argsort(key, kind='stable')].reset_index(drop=True)
    if n_rec == 0:
        frame = pd.DataFrame.from_records([])
    return _write(frame, outf, bool(regions))


def _write(df, outf, with_regions):
    """collect_mapping_info.py:165-181, the reference's own pandas calls."""
    df = df.sort_values(['qname', 'qstart'])
    bad_anchors = []
    for _, d in df.groupby('qname'):
        aln_s = list(d['aln_size'])
        bad_anchors += [1 if (aln_s[0] < 50 or aln_s[-1] < 50) else 0] * len(d)
    df['short_anchor<50bp'] = bad_anchors
    df = df.sort_values(['n_alignments', 'qname', 'qstart'], ascending=[False, True, True])
    cols = list(OUT_COLUMNS)
    if with_regions:
        cols.append('overlaps_region')
    df = df[cols]
    df.to_csv(outf, index=False, sep='\t')
    return df


def main(argv=None):
    import argparse
    import os
    ap = argparse.ArgumentParser(description='BAM (bwa + dodi) -> {name}.mappings.bed '
                                             '(reference collect_mapping_info.mapping_info)')
    ap.add_argument('--bam', required=True, help='bam file to assess')
    ap.add_argument('--out', required=True, help='output bed file')
    ap.add_argument('--regions', default=None, help='target regions (bed) for the overlaps_region column')
    ap.add_argument('--primers', default='21q1,17p6', help='comma-separated primer names of primers.csv')
    ap.add_argument('--threads', type=int, default=0)
    a = ap.parse_args(argv)
    from .main import PRIMER_SEQS
    names = a.primers.split(',')
    for p in names:
        if p not in PRIMER_SEQS:
            raise ValueError('Input primer name not in primers.csv', p, set(PRIMER_SEQS))
    mapping_info(a.bam, a.out, a.regions, {k: PRIMER_SEQS[k] for k in names}, n_threads=a.threads)
    print('Done', os.path.abspath(a.out))


if __name__ == '__main__':
    main()
