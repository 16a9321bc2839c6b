"""Hand-built ``.mappings.bed`` inputs for the edge cases the clustering path has.

Each read is a list of filling rows ``(chrom, rstart, rend, aln_size)``; two 20 bp
"bread" rows are added around them (``keep_fillings`` drops the first and last
row of every qname, cluster.py:14-31).  Cases:

* clusters whose reads carry a reversed filling (rstart > rend; prepare_data
  takes min/max, cluster.py:111-112)
* fillings inside the subtelomere mask (start < 500 kb, or < 500 kb from the
  end of a > 1 Mb chromosome; cluster.py:89-106) and on a short chromosome
  (chrM, never subtelomere-masked) and on a chromosome absent from the header
* single-row and two-row reads (all rows dropped by keep_fillings)
* qnames containing ``False`` (``--filter-false``, cluster.py:80-86)
* L=1 pairs (I=1, U=1 → edge), L=1 vs L=2 (I=1, U=2 → no edge, n_i > 0)
* the greedy-order KAT of SURVEY.md §8a A8 placed on chr7
* length/alignment-count gates (cluster.py:178-183) on both sides of the cut
* a chromosome listed in ``--cluster-mask`` (chr5)
"""
from __future__ import annotations

import numpy as np
import pandas as pd

from fslr_amd.synth import BED_COLUMNS, CHROMS, CHROM_LEN

HEADER = [(c, CHROM_LEN) for c in CHROMS] + [('chrM', 16569), ('chrY', 57_227_415)]


def _rows(qname, fillings, qgap=0, nal=None, bread=True):
    rows = []
    q = 20
    fill_rows = []
    for (c, rs, re_, aln) in fillings:
        fill_rows.append((c, rs, re_, aln, q, q + abs(aln)))
        q += abs(aln) + qgap
    n = len(fillings) + (2 if bread else 0)
    if nal is None:
        nal = n
    if bread:
        rows.append(('chr21', CHROM_LEN - 10_000, CHROM_LEN - 10_000 + 20, 20, 0, 20))
    rows.extend(fill_rows)
    if bread:
        rows.append(('chr17', CHROM_LEN - 20_000, CHROM_LEN - 20_000 + 20, 20, q, q + 20))
    out = []
    for (c, rs, re_, aln, qs, qe) in rows:
        out.append(dict(chrom=c, rstart=rs, rend=re_, qname=qname, n_alignments=nal, aln_size=aln, qstart=qs,
                        qend=qe, strand='+', mapq=60, qlen=q + 200, alignment_score=abs(aln),
                        **{'short_anchor<50bp': 1}, fslr_version='0.3.10', inferred_by_primer=0,
                        seq='ACGT' if not out else ''))
    return out


def build_edge_cases(seed: int = 5) -> pd.DataFrame:
    rng = np.random.default_rng(seed)
    reads = []
    M = 1_000_000
    # cluster A: 2 fillings, 4 reads, one with a reversed filling
    for k in range(4):
        j = int(rng.integers(-15, 16))
        f1 = ('chr1', 2 * M + j, 2 * M + 3000 + j, 3000)
        f2 = ('chr2', 5 * M + j, 5 * M + 1000 + j, 1000)
        if k == 2:
            f2 = ('chr2', 5 * M + 1000 + j, 5 * M + j, 1000)        # reversed
        reads.append((f'clA{k}.21q1F_17p6R', [f1, f2]))
    # masked: subtelomere start, near chromosome end, listed chromosome chr5
    for k in range(3):
        reads.append((f'sub{k}.21q1F_17p6R', [('chr3', 100_000 + k, 101_000 + k, 1000),
                                               ('chr4', 20 * M + k * 3, 20 * M + 2000 + k * 3, 2000)]))
        reads.append((f'end{k}.21q1F_17p6R', [('chr3', CHROM_LEN - 300_000 + k, CHROM_LEN - 299_000 + k, 1000)]))
        reads.append((f'c5_{k}.21q1F_17p6R', [('chr5', 30 * M + k, 30 * M + 2500 + k, 2500),
                                              ('chr6', 40 * M + k, 40 * M + 1500 + k, 1500)]))
    # short chromosome (not subtelomere-masked) and a chromosome absent from the header
    for k in range(3):
        reads.append((f'mito{k}.21q1F_17p6R', [('chrM', 1000 + k, 2000 + k, 1000)]))
        reads.append((f'unk{k}.21q1F_17p6R', [('chrUn_x', 100 + k, 900 + k, 800)]))
    # single-row and two-row reads
    reads.append(('solo.21q1F_17p6R', None))
    reads.append(('duo.21q1F_17p6R', 'duo'))
    # False-labelled reads forming a cluster
    for k in range(3):
        reads.append((f'fl{k}.False_17p6R', [('chr8', 60 * M + k, 60 * M + 4000 + k, 4000),
                                             ('chr9', 61 * M + k, 61 * M + 4000 + k, 4000)]))
    # L=1 vs L=1 (edge) and L=1 vs L=2 (I=1,U=2: no edge)
    reads.append(('one_a.21q1F_17p6R', [('chr10', 70 * M, 70 * M + 2000, 2000)]))
    reads.append(('one_b.21q1F_17p6R', [('chr10', 70 * M + 10, 70 * M + 2010, 2000)]))
    reads.append(('two_c.21q1F_17p6R', [('chr10', 70 * M + 5, 70 * M + 2005, 2000),
                                        ('chr11', 71 * M, 71 * M + 900, 900)]))
    # greedy-order KAT
    base = 10 * M
    reads.append(('kat_a.21q1F_17p6R', [('chr7', base - 10, base + 90, 100), ('chr7', base + 10, base + 110, 100)]))
    reads.append(('kat_b.21q1F_17p6R', [('chr7', base, base + 100, 100), ('chr7', base + 20, base + 120, 100)]))
    # length / alignment-count gates: same intervals, qlen2 differs by > 4 %; nal equal or not
    for k, (gap, nal) in enumerate([(0, None), (400, None), (400, 9), (0, 9)]):
        f = [('chr12', 80 * M + k, 80 * M + 3000 + k, 3000), ('chr13', 81 * M + k, 81 * M + 3000 + k, 3000)]
        reads.append((f'gate{k}.21q1F_17p6R', (f, gap, nal)))
    # reciprocal-overlap boundary: 5000 bp vs 4000 bp inside it (0.8 exactly) and 3999 bp (< 0.8)
    reads.append(('ro_a.21q1F_17p6R', [('chr14', 90 * M, 90 * M + 5000, 5000)]))
    reads.append(('ro_b.21q1F_17p6R', [('chr14', 90 * M + 500, 90 * M + 4500, 4000)]))
    reads.append(('ro_c.21q1F_17p6R', [('chr14', 90 * M + 501, 90 * M + 4500, 3999)]))
    # random background on chr15..chr16
    for k in range(40):
        L = int(rng.integers(1, 5))
        f = []
        for _ in range(L):
            c = f'chr{int(rng.integers(15, 17))}'
            s = int(rng.integers(2 * M, 3 * M))
            ln = int(rng.integers(300, 5000))
            f.append((c, s, s + ln, ln))
        reads.append((f'bg{k:02d}.21q1F_17p6R', f))

    rows = []
    for name, spec in reads:
        if spec is None:
            rows += [dict(chrom='chr18', rstart=5 * M, rend=5 * M + 500, qname=name, n_alignments=1, aln_size=500,
                          qstart=0, qend=500, strand='+', mapq=60, qlen=700, alignment_score=500,
                          **{'short_anchor<50bp': 0}, fslr_version='0.3.10', inferred_by_primer=0, seq='ACGT')]
        elif spec == 'duo':
            rows += _rows(name, [], nal=2)
        elif isinstance(spec, tuple):
            f, gap, nal = spec
            rows += _rows(name, f, qgap=gap, nal=nal)
        else:
            rows += _rows(name, spec)
    df = pd.DataFrame(rows)[BED_COLUMNS]
    # collect_mapping_info.py:174 order
    df = df.sort_values(['n_alignments', 'qname', 'qstart'], ascending=[False, True, True], kind='stable')
    return df.reset_index(drop=True)
