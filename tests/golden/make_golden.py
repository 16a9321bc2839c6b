"""Generate the committed golden fixtures by running the REFERENCE fslr in this container.

    python tests/golden/make_golden.py            # regenerate everything

Runs only where /root/reference exists (never on the GPU box).  The reference is
imported through ``refharness`` (stand-ins for the absent pysam / superintervals /
skbio).  Only DATA is written under tests/golden/: inputs, the
reference's outputs, and per-stage vectors.

Fixture directory layout (``tests/golden/<name>/``):
  input.mappings.bed.gz        the .mappings.bed given to ``fslr --skip-alignment``
  input.bwa_dodi.bam           header-only BAM (chromosome lengths)
  expected.cluster.bed.gz      reference {name}.mappings.cluster.bed (absent if none written)
  expected.representative.bed.gz
  meta.json                    CLI args, exit status, exception, stdout, per-stage stats
                               (``input_from``: fixture whose input files this one reuses)
  stage.json.gz                reference intermediates: ``edges`` (match_df rows, sorted),
                               ``components`` (get_subgraphs order), ``data_order``
                               (the prepare_data list: [qname, start, end])

Plus ``kats.json.gz`` (predicate known-answer tests) and ``vectors/*.npz`` (larger
synthetic cluster-id vectors regenerated from the seeded generator by the tests).
"""
from __future__ import annotations

import gzip
import hashlib
import json
import os
import shutil
import sys
import tempfile

import numpy as np
import pandas as pd

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

import refharness  # noqa: E402
from edge_cases import HEADER as EDGE_HEADER, build_edge_cases  # noqa: E402
from fslr_amd import bam_header, synth  # noqa: E402

NAME = 'fx'


def _gz_copy(src, dst):
    with open(src, 'rb') as fi, gzip.GzipFile(dst, 'wb', mtime=0) as fo:
        shutil.copyfileobj(fi, fo)


def _cli_argv_to_stage_kwargs(args):
    kw = dict(overlap=0.8, cutoffs=(1, 1, 0.66, 0.66, 0.66, 0.5), qlen_diff=0.04, n_aln_diff=0.25,
              cluster_mask=('subtelomere',), filter_false=False)
    it = iter(args)
    for a in it:
        if a == '--overlap':
            kw['overlap'] = float(next(it))
        elif a == '--jaccard-cutoffs':
            kw['cutoffs'] = tuple(float(x) for x in next(it).split(','))
        elif a == '--qlen-diff':
            kw['qlen_diff'] = float(next(it))
        elif a == '--n-alignment-diff':
            kw['n_aln_diff'] = float(next(it))
        elif a == '--cluster-mask':
            kw['cluster_mask'] = tuple(next(it).split(','))
        elif a == '--filter-false':
            kw['filter_false'] = True
    return kw


def make_fixture(name, bed_df, header, args=(), note='', input_from=None):
    out_dir = os.path.join(HERE, name)
    if os.path.isdir(out_dir):
        shutil.rmtree(out_dir)
    os.makedirs(out_dir, exist_ok=True)
    with tempfile.TemporaryDirectory() as td:
        bed_path = os.path.join(td, f'{NAME}.mappings.bed')
        bam_path = os.path.join(td, f'{NAME}.bwa_dodi.bam')
        bed_df.to_csv(bed_path, sep='\t', index=False)
        bam_header.write_bam_header(bam_path, header)
        meta = dict(name=name, args=list(args), note=note)
        if input_from is None:
            _gz_copy(bed_path, os.path.join(out_dir, 'input.mappings.bed.gz'))
            shutil.copy(bam_path, os.path.join(out_dir, 'input.bwa_dodi.bam'))
        else:
            meta['input_from'] = input_from
        # stage run (intermediates) before the CLI run so the outputs are untouched
        kw = _cli_argv_to_stage_kwargs(list(args))
        stage = {}
        try:
            st = refharness.run_stages(bed_path, bam_path, **kw)
            md = st['match_df']
            edges = sorted([[str(a), str(b), float(j)] for a, b, j in md.itertuples(index=False)])
            comps = [sorted(map(str, c)) for c in st['subgraphs']]
            meta['stage'] = dict(n_edges=len(edges), n_components=len(comps), n_data=len(st['data']))
            stage['edges'] = edges
            stage['components'] = comps
            stage['data_order'] = [[d.qname, int(d.start), int(d.end)] for d in st['data']]
            # forward degree per query read (edges added in the query's own loop)
            fwd = {}
            for a, _, _ in md.itertuples(index=False):
                fwd[a] = fwd.get(a, 0) + 1
            meta['stage']['max_fwd'] = max(fwd.values()) if fwd else 0
        except ZeroDivisionError as e:
            meta['stage_exception'] = f'{type(e).__name__}: {e}'
        res = refharness.run_cli(td, NAME, list(args))
        meta['exit_code'] = res.exit_code
        meta['stdout'] = res.output
        meta['exception'] = None if res.exception is None or isinstance(res.exception, SystemExit) else \
            f'{type(res.exception).__name__}: {res.exception}'
        for src, dst in ((f'{NAME}.mappings.cluster.bed', 'expected.cluster.bed.gz'),
                         (f'{NAME}.mappings.representative.bed', 'expected.representative.bed.gz')):
            p = os.path.join(td, src)
            dpath = os.path.join(out_dir, dst)
            if os.path.exists(p):
                _gz_copy(p, dpath)
                meta.setdefault('outputs', []).append(dst)
            elif os.path.exists(dpath):
                os.remove(dpath)
    with open(os.path.join(out_dir, 'meta.json'), 'w') as fh:
        json.dump(meta, fh, indent=1)
    if stage:
        with gzip.GzipFile(os.path.join(out_dir, 'stage.json.gz'), 'wb', mtime=0) as fh:
            fh.write(json.dumps(stage).encode())
    print(name, 'exit', meta['exit_code'], meta.get('exception'), meta.get('stage', {}))


def synth_df(n, lmax, seed, **kw):
    s = synth.generate(n, lmax, seed, **kw)
    return s.to_dataframe(), list(s.chrom_lengths.items())


def ties_df():
    """Force start ties across and within reads (pandas quicksort tie order matters)."""
    df, hdr = synth_df(600, 4, 21)
    fill = df['aln_size'] != 20
    st = df.loc[fill, 'rstart'].to_numpy()
    df.loc[fill, 'rstart'] = (st // 2000) * 2000          # coarse grid → many equal starts
    df.loc[fill, 'rend'] = df.loc[fill, 'rstart'] + df.loc[fill, 'aln_size']
    return df, hdr


def zerodiv_df():
    df, hdr = synth_df(60, 3, 4)
    fill = df.index[df['aln_size'] != 20]
    df.loc[fill[4], 'aln_size'] = 0          # a filling with aln_size 0 that overlaps its mates
    return df, hdr


def noclusters_df():
    df, hdr = synth_df(40, 3, 9, cluster_cap=1)
    return df, hdr


def chroms115_df():
    """115 chromosome names (chr1..chr22, chrX and 92 unplaced-contig-style names): the multi-GPU
    chromosome filter beyond 64 chromosomes (fslr --gpus N), and the radix-pass index build."""
    df, hdr = synth_df(1500, 8, 31)
    names = [f'chr{i}' for i in range(1, 23)] + ['chrX'] + [f'chrUn_KI2707{k:02d}v1' for k in range(92)]
    # every row keeps its coordinates; its chromosome becomes one of 115 by (chromosome, 30-Mb bin)
    base = pd.factorize(df['chrom'], sort=True)[0]
    slot = (base * 5 + (df['rstart'].to_numpy() // 30_000_000) % 5) % len(names)
    df['chrom'] = np.asarray(names, dtype=object)[slot]
    length = dict(hdr)[hdr[0][0]]
    return df, [(c, length) for c in names]


def longcap_df():
    """Dense long reads: events of up to 30 reads with 60-150 fillings, so reads of more than 64
    intervals have more than edge_threshold forward partners and the cap binds with them."""
    return synth_df(240, 150, 23, lmin=60, cluster_cap=30, size_p=0.06)


def longzero_df():
    """Long reads (65-120 fillings) where one read's qlen2 is 0 for a pair of such reads: the
    reference raises ZeroDivisionError in different_lengths_or_alignments (cluster.py:178-183)."""
    df, hdr = synth_df(60, 120, 29, lmin=65)
    q = df['qname'].to_numpy()
    rows = np.flatnonzero(np.isin(q, pd.unique(q)[:6]))     # the first reads (events are consecutive)
    df.loc[rows, 'qstart'] = 0                               # fillings span nothing: qlen2 = 0
    df.loc[rows, 'qend'] = 0
    return df, hdr


ZDCAP_ARGS = ['--n-alignment-diff', '1']


def _zero_qlen(df, qnames):
    """qlen2 = max(qend) - min(qstart) over a read's fillings (cluster.py:26-29): 0 for these reads."""
    rows = df['qname'].isin(list(qnames))
    df.loc[rows, 'qstart'] = 0
    df.loc[rows, 'qend'] = 0
    return df


def zdcap_search(limit=400):
    """Inputs where the edge cap binds and two overlapping reads both have qlen2 0, so their pair raises
    ZeroDivisionError in different_lengths_or_alignments (cluster.py:179) — but only if a loop reaches
    it (:205-209, 223-224).  With --n-alignment-diff 1 every other pair passes the gate on n_alignments,
    so zeroing the two reads' qlen2 changes nothing else.  Candidates: E* edges (a, b) whose reads both
    have more forward edges than the cap (both in the replay's T), in rank order; the oracle's reference
    loop (pinned to the reference by every other fixture) says whether it raises.  Returns the first
    pair that does not raise (both loops break before it) and the first that does."""
    sys.path.insert(0, REPO)
    from oracle import oracle as O
    base, hdr = synth_df(1500, 6, 19, cluster_cap=40, size_p=1.0 / 14)
    lens = dict(hdr)
    cut = (1, 1, 0.66, 0.66, 0.66, 0.5)
    csr, _ = O.restate_prep(base.copy(), lens, 'subtelomere', False)
    e = O.run_core(csr, 0.8, cut, 0.04, 1.0, 10, use_cap=False)
    fwd = e['fwd']
    cands = [(int(a), int(b)) for a, b in zip(e['edge_a'], e['edge_b']) if fwd[a] >= 12 and fwd[b] >= 12]
    found = {}
    for a, b in sorted(cands)[:limit]:
        qa, qb = csr.qnames[a], csr.qnames[b]
        df = _zero_qlen(base.copy(), (qa, qb))
        c2, _ = O.restate_prep(df.copy(), lens, 'subtelomere', False)
        try:
            O.run_core(c2, 0.8, cut, 0.04, 1.0, 10, use_cap=True)
            kind = 'skip'
        except ZeroDivisionError:
            kind = 'raise'
        found.setdefault(kind, (df, (qa, qb)))
        if len(found) == 2:
            break
    return found, hdr


def add_isolated_long_read(df, hdr, n_fill=70):
    """One read of n_fill fillings (more than the 64-interval chunk) far from every other interval, one
    filling with aln_size 0: the input then takes the long-read general path (no pair is evaluated with
    it: its intervals only hit its own)."""
    chrom, length = hdr[0]
    lo, hi = 600_000, 600_000 + 3000 * (n_fill + 2)
    on = df['chrom'] == chrom
    assert not ((df.loc[on, 'rend'] >= lo) & (df.loc[on, 'rstart'] <= hi)).any()
    rows = []
    tmpl = df.iloc[1].to_dict()
    for k in range(n_fill + 2):
        r = dict(tmpl)
        r.update(chrom=chrom, rstart=lo + 3000 * k, rend=lo + 3000 * k + 1000, qname='zz_isolated_long_read',
                 n_alignments=n_fill + 2, aln_size=0 if k == 5 else 1000, qstart=100 * k, qend=100 * k + 90,
                 alignment_score=1000, qlen=100 * (n_fill + 2))
        rows.append(r)
    return pd.concat([df, pd.DataFrame(rows, columns=df.columns)], ignore_index=True)


def make_round5():
    found, hdr = zdcap_search()
    for kind in ('skip', 'raise'):
        df, pair = found[kind]
        note = (f'edge cap binds; reads {pair[0]} and {pair[1]} both have qlen2 0 and overlap: their pair raises '
                f'ZeroDivisionError only if a loop reaches it ({"both loops break before it" if kind == "skip" else "a loop reaches it"})')
        make_fixture(f'zdcap_{kind}', df, hdr, args=ZDCAP_ARGS, note=note)
        make_fixture(f'zdcap_{kind}_long', add_isolated_long_read(df, hdr), hdr, args=ZDCAP_ARGS,
                     note=note + '; plus an isolated long read with an aln_size 0 filling (the general path)')


def make_kats(n_random=3000, seed=17):
    """Known answers of the reference predicates on random + boundary inputs."""
    cluster, _ = refharness.load()
    rng = np.random.default_rng(seed)
    l2c = np.zeros(100000)
    It = cluster.IntervalItem
    kats = dict(jaccard=[], lengths=[], overlap=[], cutoff=[])

    def item(c, s, e, a):
        return It(c, s, e, a, 'q', 3, 100, 0, 0)

    # overall_jaccard_similarity on random small lists (cluster.py:140-170)
    for _ in range(n_random):
        la, lb = int(rng.integers(1, 7)), int(rng.integers(1, 7))
        pct = float(rng.choice([0.8, 0.5, 0.0, 0.95, 1.0, -0.5]))
        base = int(rng.integers(0, 2000))

        def mk(L):
            out = []
            for _ in range(L):
                c = int(rng.integers(1, 3))
                s = base + int(rng.integers(0, 400))
                e = s + int(rng.integers(1, 300))
                a = int(rng.integers(max(1, (e - s) // 2), (e - s) * 2 + 2))
                out.append((c, s, e, a))
            return sorted(out, key=lambda t: t[1])
        A, B = mk(la), mk(lb)
        j, ni = cluster.overall_jaccard_similarity([item(*t) for t in A], [item(*t) for t in B], l2c, pct, 0.5)
        kats['jaccard'].append(dict(a=A, b=B, pct=pct, j=float(j), n_i=int(ni)))
    # the SURVEY §8a A8 KAT, both list orders
    A = [(1, -10, 90, 100), (1, 10, 110, 100)]
    B = [(1, 0, 100, 100), (1, 20, 120, 100)]
    for a, b in ((A, B), (A[::-1], B), (B, A)):
        j, ni = cluster.overall_jaccard_similarity([item(*t) for t in a], [item(*t) for t in b], l2c, 0.8, 0.5)
        kats['jaccard'].append(dict(a=a, b=b, pct=0.8, j=float(j), n_i=int(ni)))
    # zero aln_size raises
    for a, b in (([(1, 0, 100, 0)], [(1, 0, 100, 100)]), ([(1, 0, 100, 100)], [(2, 0, 100, 0)])):
        try:
            j, ni = cluster.overall_jaccard_similarity([item(*t) for t in a], [item(*t) for t in b], l2c, 0.8, 0.5)
            kats['jaccard'].append(dict(a=a, b=b, pct=0.8, j=float(j), n_i=int(ni)))
        except ZeroDivisionError:
            kats['jaccard'].append(dict(a=a, b=b, pct=0.8, raises='ZeroDivisionError'))
    # calculate_overlap >= pct at the floating-point boundary (cluster.py:133-136)
    for _ in range(n_random):
        a1 = int(rng.integers(1, 100000))
        a2 = int(rng.integers(1, 100000))
        pct = float(rng.choice([0.8, 0.66, 0.9, 0.1, 0.3333333333333333, 0.7, float(rng.random())]))
        t = int(np.ceil(pct * max(a1, a2))) + int(rng.integers(-2, 3))
        o = max(0, t)
        i1 = It(1, 0, o, a1, 'q', 3, 1, 0, 0)
        i2 = It(1, 0, o + int(rng.integers(0, 5)), a2, 'q', 3, 1, 0, 0)
        r = cluster.calculate_overlap(i1, i2)
        kats['overlap'].append(dict(o=o, a1=a1, a2=a2, pct=pct, ok=bool(r >= pct), end2=i2.end))
    # different_lengths_or_alignments (cluster.py:178-183) incl. boundaries and zero cases
    cases = []
    for _ in range(n_random):
        q1 = int(rng.integers(0, 20000))
        r = float(rng.choice([0.96, 0.95, 0.97, 0.959999, 1.0]))
        q2 = int(round(q1 * r)) + int(rng.integers(-1, 2))
        n1 = int(rng.integers(0, 20))
        n2 = int(rng.integers(0, 20))
        qd = float(rng.choice([0.04, 0.1, 0.0, 0.5]))
        nd = float(rng.choice([0.25, 0.0, 0.5, 1.0]))
        cases.append((q1, q2, n1, n2, qd, nd))
    cases += [(0, 0, 3, 3, 0.04, 0.25), (100, 96, 3, 4, 0.04, 0.25), (100, 95, 4, 3, 0.04, 0.25),
              (100, 95, 4, 4, 0.04, 0.25), (-5, 0, 3, 3, 0.04, 0.25), (100, 50, 0, 0, 0.04, 0.25),
              (25, 24, 3, 4, 0.04, 0.25)]
    for q1, q2, n1, n2, qd, nd in cases:
        a = item(1, 0, 1, 1)._replace(qlen2=q1, n_alignments=n1)
        b = item(1, 0, 1, 1)._replace(qlen2=q2, n_alignments=n2)
        try:
            r = cluster.different_lengths_or_alignments(a, b, qd, nd)
            kats['lengths'].append(dict(q1=q1, q2=q2, n1=n1, n2=n2, qd=qd, nd=nd, differ=bool(r)))
        except ZeroDivisionError:
            kats['lengths'].append(dict(q1=q1, q2=q2, n1=n1, n2=n2, qd=qd, nd=nd, raises='ZeroDivisionError'))
    # Jaccard cut lookup + compare (cluster.py:216-219) for I<=64, U<=128
    for cut in ([1, 1, 0.66, 0.66, 0.66, 0.5], [0.5], [1, 0.75, 0.3333333333333333]):
        table = []
        for I in range(1, 65):
            row = []
            for U in range(I, 129):
                target = cut[I - 1] if I - 1 < len(cut) else cut[-1]
                row.append(1 if I / U >= target else 0)
            table.append(row)
        kats['cutoff'].append(dict(cutoffs=cut, pass_table=table))
    with gzip.GzipFile(os.path.join(HERE, 'kats.json.gz'), 'wb', mtime=0) as fh:
        fh.write(json.dumps(kats).encode())
    print('kats', {k: len(v) for k, v in kats.items()})


def bed_digest(df):
    h = hashlib.sha256(df.to_csv(sep='\t', index=False).encode()).hexdigest()
    return h


def make_vector(name, n, lmax, seed, **kw):
    """Cluster-id vector of a larger synthetic input, from the reference stages."""
    vdir = os.path.join(HERE, 'vectors')
    os.makedirs(vdir, exist_ok=True)
    s = synth.generate(n, lmax, seed, **kw)
    df = s.to_dataframe()
    with tempfile.TemporaryDirectory() as td:
        bed_path = os.path.join(td, 'v.mappings.bed')
        bam_path = os.path.join(td, 'v.bwa_dodi.bam')
        df.to_csv(bed_path, sep='\t', index=False)
        bam_header.write_bam_header(bam_path, s.chrom_lengths.items())
        st = refharness.run_stages(bed_path, bam_path)
    names = [f"{s.name_prefix}{i:08d}{s.name_suffix}" for i in range(s.n_reads)]
    idx = {q: i for i, q in enumerate(names)}
    comp = np.full(s.n_reads, -1, np.int32)
    for c, members in enumerate(st['subgraphs']):
        for q in members:
            comp[idx[q]] = c
    md = st['match_df']
    fwd = np.zeros(s.n_reads, np.int32)
    for a in md['query1']:
        fwd[idx[a]] += 1
    np.savez_compressed(os.path.join(vdir, f'{name}.npz'), comp=comp, fwd=fwd,
                        params=np.array([n, lmax, seed], np.int64), n_edges=np.int64(len(md)),
                        digest=np.array(bed_digest(df)))
    print('vector', name, 'edges', len(md), 'components', len(st['subgraphs']), 'max_fwd', int(fwd.max()))


def make_longreads():
    # reads of more than 64 fillings: the device splits them into chunks
    df, hdr = synth_df(400, 150, 21, lmin=1)
    make_fixture('longreads_400', df, hdr, note='1-150 fillings: reads beyond the 64-interval chunk width')


def make_round3():
    df, hdr = chroms115_df()
    make_fixture('chroms_115', df, hdr, note='115 chromosome names: --gpus N beyond 64 chromosomes')
    df, hdr = longcap_df()
    make_fixture('longcap_240', df, hdr, note='dense reads of 60-150 fillings: the edge cap binds with long reads')
    make_fixture('longreads_p0', *synth_df(160, 110, 37, lmin=50), args=['--overlap', '0', '--jaccard-cutoffs', '0.2'],
                 note='long reads with overlap 0 (matches need not overlap; the walk engine)')
    df, hdr = longzero_df()
    make_fixture('longzero_60', df, hdr, note='a long read with qlen2 0 raises ZeroDivisionError')


def main():
    sys.stdout.reconfigure(line_buffering=True)
    refharness.load()
    if sys.argv[1:] == ['--only', 'longreads_400']:
        make_longreads()
        return
    if sys.argv[1:2] == ['--round3']:
        make_round3()
        return
    if sys.argv[1:2] == ['--round5']:
        make_round5()
        return
    df, hdr = synth_df(1000, 3, 0, lmin=3)
    make_fixture('cfg1_1k_x3', df, hdr, note='BASELINE config 1: 1k reads x 3 fillings, defaults')
    df, hdr = synth_df(2000, 8, 7)
    make_fixture('mixed_2k_l8', df, hdr, note='cfg2 shape, 2k reads, 1-8 fillings, defaults')
    make_fixture('params_a', df, hdr, input_from='mixed_2k_l8', args=['--overlap', '0.5', '--jaccard-cutoffs', '1,0.5,0.5',
                                            '--qlen-diff', '0.1', '--n-alignment-diff', '0.5'])
    make_fixture('params_b', df, hdr, input_from='mixed_2k_l8', args=['--overlap', '0.95', '--jaccard-cutoffs', '0.3',
                                            '--qlen-diff', '0.0', '--n-alignment-diff', '0.0'])
    make_fixture('params_nomask', df, hdr, input_from='mixed_2k_l8', args=['--cluster-mask', ''])
    df, hdr = synth_df(1500, 16, 3)
    make_fixture('mixed_1500_l16', df, hdr, note='cfg3 shape, 1500 reads, 1-16 fillings')
    df, hdr = synth_df(800, 64, 13, dist='zipf')
    make_fixture('zipf_800_l64', df, hdr, note='cfg5 shape: truncated Zipf 1-64 fillings')
    edf = build_edge_cases()
    make_fixture('edge_cases', edf, EDGE_HEADER, note='hand-built edge cases (tests/golden/edge_cases.py)')
    make_fixture('edge_cases_ff', edf, EDGE_HEADER, input_from='edge_cases', args=['--filter-false', '--cluster-mask',
                                                          'chr5,subtelomere,chrNotThere'])
    make_fixture('edge_cases_p0', edf, EDGE_HEADER, input_from='edge_cases', args=['--overlap', '0', '--jaccard-cutoffs', '0.2'],
                 note='overlap 0: every same-chrom pair matches, candidates gated by index overlap')
    df, hdr = ties_df()
    make_fixture('ties_600', df, hdr, note='many equal starts: pandas quicksort tie order (host-side)')
    df, hdr = zerodiv_df()
    make_fixture('zerodiv', df, hdr, note='aln_size 0 on an evaluated filling raises ZeroDivisionError')
    df, hdr = noclusters_df()
    make_fixture('noclusters', df, hdr, note='no edges: "No clusters were found." and no output files')
    df, hdr = synth_df(1500, 6, 19, cluster_cap=40, size_p=1.0 / 14)
    make_fixture('capbind_1500', df, hdr, note='clusters up to 40 reads: edge cap binds (stub-order)')
    make_longreads()
    make_round3()
    make_round5()
    make_kats()
    make_vector('v10k_l8_s7', 10_000, 8, 7)
    make_vector('v20k_l16_s11', 20_000, 16, 11)


if __name__ == '__main__':
    main()
