"""Pin the CPU oracle (oracle/) to the reference's own outputs (tests/golden/).

The oracle is only trusted as a checker after it reproduces every committed
golden vector: per-predicate KATs, the prepare_data order, the edge list, the
component order and the final cluster ids of every fixture (CPU only).
"""
import os

import numpy as np
import pandas as pd
import pytest

import fixtures as fx
from fslr_amd import bam_header, synth
from oracle import oracle as O

CLUSTER_FIXTURES = [f for f in fx.FIXTURES]


def _oracle_run(name):
    kw = fx.cli_options(name)
    bed = fx.input_bed(name)
    lens = bam_header.get_chromosome_lengths(fx.input_bam(name))
    csr, bed2 = O.restate_prep(bed, lens, kw['cluster_mask'], kw['filter_false'])
    cut = [float(x) for x in kw['jaccard_cutoffs'].split(',')]
    res = O.run_core(csr, kw['overlap'], cut, kw['qlen_diff'], kw['n_alignment_diff'], 10, use_cap=True)
    return csr, bed2, res


@pytest.mark.parametrize('name', CLUSTER_FIXTURES)
def test_oracle_reproduces_reference_fixture(name):
    meta = fx.meta(name)
    if meta.get('exception'):
        assert 'ZeroDivisionError' in meta['exception']
        with pytest.raises(ZeroDivisionError):
            _oracle_run(name)
        return
    csr, bed2, res = _oracle_run(name)
    st = fx.stage(name)
    # prepare_data order (cluster.py:109-121) — ties included
    data = sorted(range(len(csr.data_pos)), key=lambda k: csr.data_pos[k])
    read_of = np.repeat(np.arange(csr.n_reads), np.diff(csr.read_off))
    mine = [[csr.qnames[read_of[k]], int(csr.start[k]), int(csr.end[k])] for k in data]
    assert mine == st['data_order']
    # edge list (match_df) with the exact Python float jaccard
    edges = sorted([csr.qnames[a], csr.qnames[b], I / U]
                   for a, b, I, U in zip(res['edge_a'], res['edge_b'], res['edge_I'], res['edge_U']))
    assert edges == [[a, b, j] for a, b, j in st['edges']]
    # components in get_subgraphs order
    comps = {}
    for r, c in enumerate(res['comp']):
        if c >= 0:
            comps.setdefault(int(c), []).append(csr.qnames[r])
    assert [sorted(comps[c]) for c in range(len(comps))] == st['components']
    # final cluster ids (main.py:247-342)
    num = O.restate_numbering(bed2, csr, res['comp'])
    text = fx.expected_text(name, 'cluster')
    if num is None:
        assert text is None and 'No clusters were found.' in meta['stdout']
        return
    ids, kind = num
    gold = pd.read_csv(fx.os.path.join(fx.GOLDEN, name, 'expected.cluster.bed.gz'), sep='\t')
    assert (gold['cluster'].dtype.kind == 'f') == (kind == 'float')
    for q, c, n in zip(gold['qname'], gold['cluster'], gold['n_reads']):
        assert ids[q] == (c, n)
    assert res['stats']['max_fwd'] == meta['stage']['max_fwd']


def test_kat_jaccard():
    for k in fx.kats()['jaccard']:
        if 'raises' in k:
            with pytest.raises(ZeroDivisionError):
                O.jaccard_lists(k['a'], k['b'], k['pct'])
            continue
        I, U = O.jaccard_lists(k['a'], k['b'], k['pct'])
        assert I == k['n_i']
        assert (I / U if U else 0) == k['j']


def test_kat_jaccard_symmetric():
    """First-fit greedy count is symmetric — the GPU evaluates B-major."""
    for k in fx.kats()['jaccard']:
        if 'raises' in k:
            continue
        assert O.jaccard_lists(k['b'], k['a'], k['pct'])[0] == k['n_i']


def test_kat_lengths():
    for k in fx.kats()['lengths']:
        args = (k['q1'], k['q2'], k['n1'], k['n2'], k['qd'], k['nd'])
        if 'raises' in k:
            with pytest.raises(ZeroDivisionError):
                O.lengths_differ(*args)
        else:
            assert O.lengths_differ(*args) == k['differ']


def test_kat_overlap():
    for k in fx.kats()['overlap']:
        I, _ = O.jaccard_lists([(1, 0, k['o'], k['a1'])], [(1, 0, k['end2'], k['a2'])], k['pct'])
        assert bool(I) == k['ok']


@pytest.mark.parametrize('vec', ['v10k_l8_s7', 'v20k_l16_s11'])
def test_oracle_vectors(vec):
    z = np.load(os.path.join(fx.GOLDEN, 'vectors', f'{vec}.npz'))
    n, lmax, seed = (int(x) for x in z['params'])
    s = synth.generate(n, lmax, seed)
    df = s.to_dataframe()
    from make_golden import bed_digest
    assert bed_digest(df) == str(z['digest']), 'synthetic generator drifted from the committed vector'
    csr, _ = O.restate_prep(df, s.chrom_lengths)
    res = O.run_core(csr)
    names = [f"{s.name_prefix}{i:08d}{s.name_suffix}" for i in range(s.n_reads)]
    idx = {q: i for i, q in enumerate(names)}
    comp = np.full(s.n_reads, -1, np.int32)
    fwd = np.zeros(s.n_reads, np.int32)
    for r, q in enumerate(csr.qnames):
        comp[idx[q]] = res['comp'][r]
        fwd[idx[q]] = res['fwd'][r]
    np.testing.assert_array_equal(comp, z['comp'])
    np.testing.assert_array_equal(fwd, z['fwd'])
    assert res['stats']['n_edges'] == int(z['n_edges'])


@pytest.mark.parametrize('nthreads', [1, 4])
def test_threaded_cpu_baseline_counts_equal_the_oracle(nthreads):
    """bench.py's all-core CPU baseline (oracle_count_threads) evaluates exactly the pairs of the
    uncapped reference loop; a block-strided sample evaluates the sampled reads' forward pairs."""
    from fslr_amd import synth
    s = synth.generate(20_000, 16, 11)
    csr = s.interval_data().csr()
    cnt = np.diff(csr.read_off)
    oc = O.OracleCSR(csr.read_off, csr.iv_chrom, csr.iv_start, csr.iv_end, csr.iv_aln, np.repeat(csr.read_qlen2, cnt),
                     np.repeat(csr.read_nal, cnt), csr.data_pos)
    full = O.run_core(oc, use_cap=False)
    got = O.count_threads(oc, nthreads=nthreads)
    for k in ('evaluated_pairs', 'jaccard_evals', 'n_edges'):
        assert got[k] == full['stats'][k], k
    # stride 4: query reads of blocks 0, 4, 8, ... == forward edges of those reads in the full run
    part = O.count_threads(oc, nthreads=nthreads, stride=4)
    own = (np.arange(csr.n_reads) // 64) % 4 == 0
    assert part['n_edges'] == int(full['fwd'][own].sum())


def _dense_oracle_csr(n, lmax, seed, squeeze, ccap):
    import dataclasses
    s = synth.generate(n, lmax, seed, cluster_cap=ccap, size_p=0.05)
    c = s.interval_data().csr()
    st = c.iv_start.astype(np.int64) // squeeze
    en = st + (c.iv_end.astype(np.int64) - c.iv_start)
    c = dataclasses.replace(c, iv_start=st.astype(np.int32), iv_end=en.astype(np.int32))
    cnt = np.diff(c.read_off)
    return O.OracleCSR(c.read_off, c.iv_chrom, c.iv_start, c.iv_end, c.iv_aln, np.repeat(c.read_qlen2, cnt),
                       np.repeat(c.read_nal, cnt), c.data_pos)


@pytest.mark.parametrize('n,lmax,seed,squeeze,ccap,thr', [
    (6_000, 16, 47, 100, 30, 3),
    (4_000, 8, 53, 2000, 10, 1),
    (4_000, 8, 59, 50, 200, 10),
    (3_000, 64, 13, 300, 40, 10),
])
def test_lean_seen_set_equals_pair_set(n, lmax, seed, squeeze, ccap, thr):
    """oracle_query_lean (the seen-set held as per-read reached lists, for the full config-5 pin) gives
    the pair-set oracle's result exactly where the cap binds for many reads."""
    oc = _dense_oracle_csr(n, lmax, seed, squeeze, ccap)
    a = O.run_core(oc, edge_threshold=thr, use_cap=True)
    b = O.run_core(oc, edge_threshold=thr, use_cap=True, lean=True)
    assert a['stats']['max_fwd'] >= thr and a['stats'] == b['stats']
    for k in ('edge_a', 'edge_b', 'edge_I', 'edge_U', 'fwd', 'comp'):
        np.testing.assert_array_equal(a[k], b[k])


@pytest.mark.parametrize('name', CLUSTER_FIXTURES)
def test_lean_seen_set_on_reference_fixtures(name):
    kw = fx.cli_options(name)
    if fx.meta(name).get('exception'):
        return
    bed = fx.input_bed(name)
    lens = bam_header.get_chromosome_lengths(fx.input_bam(name))
    csr, _ = O.restate_prep(bed, lens, kw['cluster_mask'], kw['filter_false'])
    cut = [float(x) for x in kw['jaccard_cutoffs'].split(',')]
    args = (csr, kw['overlap'], cut, kw['qlen_diff'], kw['n_alignment_diff'], 10)
    a, b = O.run_core(*args, use_cap=True), O.run_core(*args, use_cap=True, lean=True)
    assert a['stats'] == b['stats']
    for k in ('edge_a', 'edge_b', 'fwd', 'comp'):
        np.testing.assert_array_equal(a[k], b[k])
