"""GPU parity: the HIP path (through the C ABI) against the golden fixtures and the CPU oracle.

Run on a real MI355X:  python -m pytest tests -m gpu -x -q
Bar: bit-exact (integer / index work): identical edge sets with identical
I/U, identical forward degrees, identical components and cluster ids, identical
output files.
"""
import gzip
import io
import os
import shutil
import tempfile
import warnings

import numpy as np
import pandas as pd
import pytest

import fixtures as fx
from host_pipeline import host_prepare
from fslr_amd import _lib, cluster, synth
from fslr_amd.prep import fold_overlap_threshold, pass_table
from oracle import oracle as O

pytestmark = pytest.mark.gpu
# the two pair engines (fslr_hip.h FSLR_ENGINE_*): the read walk counts evaluated pairs, the
# position sweep does not; both must give the oracle's edges, degrees and components
ENGINES = ['walk', 'sweep']


@pytest.fixture(scope='module')
def ctx():
    c = _lib.Context(0)
    yield c
    c.close()


def oracle_from_csr(c):
    cnt = np.diff(c.read_off)
    return O.OracleCSR(c.read_off, c.iv_chrom, c.iv_start, c.iv_end, c.iv_aln, np.repeat(c.read_qlen2, cnt),
                       np.repeat(c.read_nal, cnt), c.data_pos)


def gpu_run(ctx, csr, overlap=0.8, cutoffs=(1, 1, 0.66, 0.66, 0.66, 0.5), qlen_diff=0.04, nal_diff=0.25,
            full_sort=False, cap=None, engine='walk'):
    """E* (every candidate pair) or, with ``cap`` = edge_threshold, the reference's capped graph."""
    thr = fold_overlap_threshold(csr.iv_aln, overlap)
    if full_sort:
        ctx.set_reads(csr.read_off, csr.read_qlen2, csr.read_nal, csr.iv_chrom, csr.iv_start, csr.iv_end, thr,
                      csr.n_chroms)
    else:
        ctx.load_csr(csr, thr)
    ctx.reserve_edges(max(1 << 16, 12 * csr.n_reads))
    ctx.build_index()
    st = ctx.run_query(1 - qlen_diff, 1 - nal_diff, pass_table(cutoffs), engine=engine)
    if engine != 'auto':
        assert st['engine'] == engine
    if cap is not None:
        st['cap'] = ctx.apply_edge_cap(cap)
        st['n_edges'] = ctx.stats()['n_edges']
        st['max_fwd'] = st['cap']['max_fwd']
    ctx.components()
    a, b, I, U = ctx.edges(st['n_edges'])
    return dict(stats=st, labels=ctx.labels(), fwd=ctx.fwd_degree(), a=a, b=b, I=I, U=U)


def compare_capped_with_oracle(g, o, n):
    """Capped graph: the same edges oriented as (read whose loop formed it, partner), the same
    edges-per-loop counts and the same components (cluster ids) as the oracle's reference loop."""
    ge = sorted(zip(g['a'].tolist(), g['b'].tolist(), g['I'].tolist(), g['U'].tolist()))
    oe = sorted(zip(o['edge_a'].tolist(), o['edge_b'].tolist(), o['edge_I'].tolist(), o['edge_U'].tolist()))
    assert len(ge) == len(oe)
    assert ge == oe
    np.testing.assert_array_equal(g['fwd'], o['fwd'])
    assert g['stats']['max_fwd'] == o['stats']['max_fwd']
    lab = g['labels']
    sizes = np.bincount(lab, minlength=n)
    roots = np.flatnonzero(sizes >= 2)
    rid = np.full(n, -1)
    rid[roots] = np.arange(roots.size)
    np.testing.assert_array_equal(np.where(sizes[lab] >= 2, rid[lab], -1), o['comp'])


def compare_with_oracle(g, o, n):
    ge = sorted(zip(g['a'].tolist(), g['b'].tolist(), g['I'].tolist(), g['U'].tolist()))
    oe = sorted(zip(o['edge_a'].tolist(), o['edge_b'].tolist(), o['edge_I'].tolist(), o['edge_U'].tolist()))
    assert len(ge) == len(oe)
    assert ge == oe
    np.testing.assert_array_equal(g['fwd'], o['fwd'])
    if g['stats']['engine'] == 'walk':
        assert g['stats']['evaluated_pairs'] == o['stats']['evaluated_pairs']
        assert g['stats']['jaccard_evals'] == o['stats']['jaccard_evals']
    else:
        assert g['stats']['evaluated_pairs'] == -1
    assert g['stats']['max_fwd'] == o['stats']['max_fwd']
    # components: oracle numbers by first insertion (== min rank), device labels = min rank
    lab = g['labels']
    sizes = np.bincount(lab, minlength=n)
    node = sizes[lab] >= 2
    roots = np.flatnonzero(sizes >= 2)
    rid = np.full(n, -1)
    rid[roots] = np.arange(roots.size)
    comp = np.where(node, rid[lab], -1)
    np.testing.assert_array_equal(comp, o['comp'])


# ------------------------------------------------------------------ end-to-end CLI vs golden
CLI_FIXTURES = list(fx.FIXTURES)


def run_product_cli(name, tmp, io_flag='--native-io'):
    from click.testing import CliRunner
    from fslr_amd.main import pipeline
    with open(os.path.join(tmp, 'fx.mappings.bed'), 'w') as fh:
        fh.write(fx.input_bed_text(name))
    shutil.copy(fx.input_bam(name), os.path.join(tmp, 'fx.bwa_dodi.bam'))
    args = ['--name', 'fx', '--out', tmp, '--ref', 'unused.fa', '--primers', '21q1', '--skip-alignment'] + \
        fx.meta(name)['args'] + [io_flag]
    return CliRunner().invoke(pipeline, args, catch_exceptions=True)


@pytest.mark.parametrize('io_flag', ['--native-io', '--pandas-io'])
@pytest.mark.parametrize('name', CLI_FIXTURES)
def test_cli_matches_reference_outputs(name, io_flag):
    meta = fx.meta(name)
    with tempfile.TemporaryDirectory() as tmp:
        res = run_product_cli(name, tmp, io_flag)
        if meta['exception']:
            assert isinstance(res.exception, ZeroDivisionError), res.output
            return
        assert res.exit_code == 0, (res.output, res.exception)
        for which in ('cluster', 'representative'):
            want = fx.expected_text(name, which)
            path = os.path.join(tmp, f'fx.mappings.{which}.bed')
            if want is None:
                assert not os.path.exists(path)
                assert 'No clusters were found.' in res.output
            else:
                got = open(path).read()
                assert got == want, f'{name}: {which} output differs'
        assert ('fslr finished' in res.output) == ('fslr finished' in meta['stdout'])


@pytest.mark.parametrize('name', ['cfg1_1k_x3', 'capbind_1500', 'zerodiv', 'noclusters', 'longreads_400', 'params_a',
                                  'edge_cases_p0', 'zipf_800_l64', 'chroms_115', 'longcap_240', 'zdcap_skip',
                                  'zdcap_raise', 'zdcap_skip_long', 'zdcap_raise_long', 'longreads_p0',
                                  'longzero_60'])
def test_cli_multi_gpu_matches_reference_outputs(name):
    """``fslr --gpus 2``: two rank processes (sharing this box's one GPU over gloo) run the
    chromosome-split sweep, or the query-shard split where the sweep does not apply (fslr_amd.multi);
    outputs byte-identical to the reference's.  Covers the cap replay (capbind_1500), a
    ZeroDivisionError raised on every rank (zerodiv), the empty graph, overlap <= 0 (edge_cases_p0,
    longreads_p0), 115 chromosomes, long reads with and without the cap binding (longreads_400,
    longcap_240) and ZeroDivisionError pairs under a binding cap (zdcap_*)."""
    from fslr_amd import multi
    meta = fx.meta(name)
    multi.last_path = None
    with tempfile.TemporaryDirectory() as tmp:
        res = run_product_cli(name, tmp, '--gpus=2')
        # every input takes a two-rank split (no one-GPU fallback): the position split of the sweep (the
        # chromosome split beyond 64 chromosomes), or the query-shard split for overlap <= 0
        # (edge_cases_p0), aln_size == 0 (zerodiv) and long reads
        want_path = {'edge_cases_p0': 'walk', 'zerodiv': 'walk', 'longreads_400': 'long', 'longcap_240': 'long',
                     'zdcap_skip_long': 'long', 'zdcap_raise_long': 'long', 'longreads_p0': 'long',
                     'longzero_60': 'long', 'chroms_115': 'sweep-chrom'}.get(name, 'sweep-position')
        assert multi.last_path == want_path, (name, multi.last_path)
        if meta['exception']:
            assert isinstance(res.exception, ZeroDivisionError), (res.output, res.exception)
            return
        assert res.exit_code == 0, (res.output, res.exception)
        for which in ('cluster', 'representative'):
            want = fx.expected_text(name, which)
            path = os.path.join(tmp, f'fx.mappings.{which}.bed')
            if want is None:
                assert not os.path.exists(path)
                assert 'No clusters were found.' in res.output
            else:
                assert open(path).read() == want, f'{name}: {which} output differs'


@pytest.mark.parametrize('engine', ENGINES)
@pytest.mark.parametrize('name', ['zdcap_skip', 'zdcap_raise'])
def test_zero_division_under_binding_cap(ctx, name, engine):
    """Two overlapping reads with qlen2 0 (their pair raises ZeroDivisionError in
    different_lengths_or_alignments, cluster.py:179) inside a locus where the edge cap binds: the
    reference raises only if a loop reaches the pair (cluster.py:205-209, 223-224).  zdcap_skip: both
    reads' loops break before it, no raise, the capped graph is the reference's; zdcap_raise: a loop
    reaches it.  The engines list such pairs instead of raising (zd_pairs); the cap replay decides."""
    data, _, kw = host_prepare(name)
    csr = data.csr()
    cut = [float(x) for x in kw['jaccard_cutoffs'].split(',')]
    args = dict(overlap=kw['overlap'], cutoffs=cut, qlen_diff=kw['qlen_diff'], nal_diff=kw['n_alignment_diff'])
    oc = oracle_from_csr(csr)
    oargs = (kw['overlap'], cut, kw['qlen_diff'], kw['n_alignment_diff'], 10)
    if fx.meta(name)['exception']:
        with pytest.raises(ZeroDivisionError):
            O.run_core(oc, *oargs, use_cap=True)
        with pytest.raises(ZeroDivisionError):
            gpu_run(ctx, csr, cap=10, engine=engine, **args)
        return
    o = O.run_core(oc, *oargs, use_cap=True)
    g = gpu_run(ctx, csr, cap=10, engine=engine, **args)
    assert g['stats']['zd_pairs'] >= 1 and g['stats']['cap']['applied'] == 1
    compare_capped_with_oracle(g, o, csr.n_reads)
    # without the cap (every loop runs to its end) the same input raises
    with pytest.raises(ZeroDivisionError):
        gpu_run(ctx, csr, cap=10 ** 6, engine=engine, **args)


@pytest.mark.parametrize('name', [f for f in fx.FIXTURES if fx.stage(f) is not None])
def test_query_interval_trees_edges_match_reference(name):
    data, _, kw = host_prepare(name)
    cut = [float(x) for x in kw['jaccard_cutoffs'].split(',')]
    with warnings.catch_warnings():
        warnings.simplefilter('ignore', cluster.EdgeCapWarning)
        tree = cluster.build_interval_trees(data)
        match_df, G = cluster.query_interval_trees(tree, data, kw['overlap'], cut, 10, kw['qlen_diff'],
                                                   kw['n_alignment_diff'])
    got = sorted([a, b, j] for a, b, j in match_df.itertuples(index=False))
    want = fx.stage(name)['edges']
    # the reference's match set, rows (query read, partner, j) — also where the cap binds
    # (capbind_1500: max forward degree 15 > 10), edges formed in the partner's loop included
    assert got == want
    assert [sorted(c) for c in cluster.get_subgraphs(G)] == fx.stage(name)['components']


@pytest.mark.parametrize('name', ['mixed_2k_l8', 'capbind_1500'])
def test_reference_item_list_drops_in(name):
    """build_interval_trees / query_interval_trees given the reference's prepare_data output (a
    list of IntervalItem) return the same match set and components as given IntervalData."""
    data, _, kw = host_prepare(name)
    cut = [float(x) for x in kw['jaccard_cutoffs'].split(',')]
    args = (kw['overlap'], cut, 10, kw['qlen_diff'], kw['n_alignment_diff'])
    m1, G1 = cluster.query_interval_trees(cluster.build_interval_trees(data), data, *args)
    items = list(data)
    m2, G2 = cluster.query_interval_trees(cluster.build_interval_trees(items), items, *args)
    assert sorted(map(tuple, m1.itertuples(index=False))) == sorted(map(tuple, m2.itertuples(index=False)))
    assert [sorted(c) for c in cluster.get_subgraphs(G1)] == [sorted(c) for c in cluster.get_subgraphs(G2)]
    assert sorted(map(tuple, m2.itertuples(index=False))) == sorted(map(tuple, fx.stage(name)['edges']))


@pytest.mark.parametrize('engine', ENGINES)
def test_capbind_device_equals_uncapped_oracle(ctx, engine):
    data, _, _ = host_prepare('capbind_1500')
    csr = data.csr()
    g = gpu_run(ctx, csr, engine=engine)
    o = O.run_core(oracle_from_csr(csr), use_cap=False)
    compare_with_oracle(g, o, csr.n_reads)
    assert g['stats']['max_fwd'] > 10


@pytest.mark.parametrize('engine', ENGINES)
def test_capbind_device_capped_equals_reference_loop(ctx, engine):
    data, _, _ = host_prepare('capbind_1500')
    csr = data.csr()
    g = gpu_run(ctx, csr, cap=10, engine=engine)
    o = O.run_core(oracle_from_csr(csr), use_cap=True)
    assert g['stats']['cap']['applied'] == 1 and g['stats']['cap']['capped'] > 0
    compare_capped_with_oracle(g, o, csr.n_reads)


def _squeezed(n, lmax, seed, squeeze, dist='uniform', cluster_cap=10, size_p=1 / 3):
    import dataclasses
    s = synth.generate(n, lmax, seed, dist=dist, cluster_cap=cluster_cap, size_p=size_p)
    csr = s.interval_data().csr()
    st = csr.iv_start.astype(np.int64) // squeeze          # monotone: the data order stays start-sorted
    en = st + (csr.iv_end.astype(np.int64) - csr.iv_start)
    return dataclasses.replace(csr, iv_start=st.astype(np.int32), iv_end=en.astype(np.int32))


@pytest.mark.parametrize('n,lmax,seed,squeeze,dist,ccap,thr', [
    (30_000, 16, 41, 400, 'uniform', 60, 10),
    (20_000, 64, 13, 300, 'zipf', 40, 10),
    (20_000, 16, 47, 100, 'uniform', 30, 3),
    (8_000, 8, 53, 2000, 'uniform', 10, 1),
    (8_000, 8, 59, 50, 'uniform', 200, 40),
])
@pytest.mark.parametrize('engine', ENGINES)
def test_dense_capped_vs_oracle(ctx, n, lmax, seed, squeeze, dist, ccap, thr, engine):
    """Events of up to `ccap` reads (forward degrees far above the cap) on a squeezed genome: the
    cap binds for many reads, with chains of pairs left unseen by capped loops; the replayed graph
    equals the oracle's reference loop exactly."""
    csr = _squeezed(n, lmax, seed, squeeze, dist, cluster_cap=ccap, size_p=0.05)
    g = gpu_run(ctx, csr, cap=thr, engine=engine)
    o = O.run_core(oracle_from_csr(csr), edge_threshold=thr, use_cap=True)
    assert g['stats']['cap']['applied'] == 1 and g['stats']['cap']['capped'] > 0
    assert g['stats']['cap']['dropped'] > 0 or thr == 40
    compare_capped_with_oracle(g, o, csr.n_reads)


@pytest.mark.parametrize('engine', ENGINES)
@pytest.mark.parametrize('thr', [1, 10])
def test_one_locus_capped_vs_oracle(ctx, thr, engine):
    """1500 reads on one locus with runs of equal starts (the search order's tie rule decides
    which pairs a capped loop reaches)."""
    n = 1500
    off = np.arange(n + 1, dtype=np.int64)
    chrom = np.zeros(n, np.int32)
    start = np.sort(np.full(n, 5000, np.int32) + (np.arange(n) % 7).astype(np.int32))
    end = start + 1000 - (np.arange(n) % 3).astype(np.int32)
    aln = np.full(n, 1000, np.int64)
    q = np.full(n, 100, np.int32)
    m = np.full(n, 3, np.int32)
    thr_iv = fold_overlap_threshold(aln, 0.8)
    ctx.set_reads(off, q, m, chrom, start, end, thr_iv, 1, iv_data_pos=np.arange(n))
    ctx.reserve_edges(n * n)
    ctx.build_index()
    st = ctx.run_query(1 - 0.04, 1 - 0.25, pass_table([1.0]), engine=engine)
    st['cap'] = ctx.apply_edge_cap(thr)
    st['n_edges'] = ctx.stats()['n_edges']
    st['max_fwd'] = st['cap']['max_fwd']
    ctx.components()
    a, b, I, U = ctx.edges(st['n_edges'])
    g = dict(stats=st, labels=ctx.labels(), fwd=ctx.fwd_degree(), a=a, b=b, I=I, U=U)
    o = O.run_core(O.OracleCSR(off, chrom, start, end, aln, q, m, np.arange(n)), 0.8, (1.0,), 0.04, 0.25,
                   edge_threshold=thr, use_cap=True)
    compare_capped_with_oracle(g, o, n)


@pytest.mark.parametrize('n,lmax,seed,squeeze,dist,ccap', [
    (30_000, 16, 41, 400, 'uniform', 60),
    (20_000, 64, 13, 300, 'zipf', 40),
    (8_000, 8, 59, 50, 'uniform', 200),
])
def test_sweep_edges_one_run_per_lower_read(ctx, n, lmax, seed, squeeze, dist, ccap):
    """The sweep engine writes each read's forward edges E* as one run of the edge list (its edge
    stage never splits a read, reads of up to 256 forward edges), which the one-GPU cap replay walks
    (cap.hip k_cap_runs1; a split list falls back to the full-list path)."""
    csr = _squeezed(n, lmax, seed, squeeze, dist, cluster_cap=ccap, size_p=0.05)
    g = gpu_run(ctx, csr, engine='sweep')
    a = g['a']
    heads = a[np.r_[True, a[1:] != a[:-1]]]
    assert g['fwd'].max() <= 256
    assert np.unique(heads).size == heads.size          # no read starts two runs


@pytest.mark.parametrize('engine', ENGINES)
def test_cap_not_binding_is_identity(ctx, engine):
    s = synth.generate(30_000, 16, 2)
    csr = s.interval_data().csr()
    g1 = gpu_run(ctx, csr, engine=engine)
    g2 = gpu_run(ctx, csr, cap=10, engine=engine)
    assert g2['stats']['cap']['applied'] == 0
    assert sorted(zip(g1['a'], g1['b'], g1['I'])) == sorted(zip(g2['a'], g2['b'], g2['I']))
    np.testing.assert_array_equal(g1['labels'], g2['labels'])


def test_union_find_labels_stable_over_repeats(ctx):
    """Labels of the device union-find equal a host union-find over the same edges on every one of
    30 repeats (the finalize pass once raced with path halving, ~1 run in 40 on capbind_1500)."""
    from fslr_amd.dist import union_find_labels
    data, _, _ = host_prepare('capbind_1500')
    csr = data.csr()
    g = gpu_run(ctx, csr, cap=10)
    want = union_find_labels(csr.n_reads, g['a'], g['b'])
    for _ in range(30):
        ctx.components()
        np.testing.assert_array_equal(ctx.labels(), want)


def test_components_after_the_sweeps_pre_hook(ctx):
    """The sweep's pair kernel pre-hooks the union-find as it forms edges, so the next
    fslr_components runs only the unions: its labels must equal a host union-find over the stored edges,
    and so must every sequence that invalidates the hook first (a second components call, an edge sort,
    a walk query, a binding cap's rewritten edges, the local forest's pairs)."""
    from fslr_amd.dist import union_find_labels
    s = synth.generate(30_000, 16, 5)
    csr = s.interval_data().csr()
    n = csr.n_reads
    qc, nc, pt = 1 - 0.04, 1 - 0.25, pass_table([1, 1, 0.66, 0.66, 0.66, 0.5])
    ctx.load_csr(csr, fold_overlap_threshold(csr.iv_aln, 0.8))
    ctx.reserve_edges(12 * n)

    def host_labels():
        a, b, _, _ = ctx.edges(ctx.stats()['n_edges'])
        return union_find_labels(n, a, b)

    for seq in ('direct', 'twice', 'sorted', 'walk_after', 'forest'):
        ctx.build_index()
        ctx.query(qc, nc, pt, 10, engine='sweep')
        if seq == 'walk_after':
            ctx.query(qc, nc, pt, 10, engine='walk')
        if seq == 'sorted':
            ctx.sort_edges()
        if seq == 'forest':
            ctx.local_forest()
            want = host_labels()
            got = ctx.labels()
            np.testing.assert_array_equal(got, want, err_msg=seq)     # the forest finalizes the parents
            continue
        ctx.components()
        if seq == 'twice':
            ctx.components()
        np.testing.assert_array_equal(ctx.labels(), host_labels(), err_msg=seq)
    # a binding cap rewrites the edges: the components after it are those of the capped list
    data, _, _ = host_prepare('capbind_1500')
    c2 = data.csr()
    ctx.load_csr(c2, fold_overlap_threshold(c2.iv_aln, 0.8))
    ctx.reserve_edges(max(1 << 16, 12 * c2.n_reads))
    ctx.build_index()
    ctx.query(qc, nc, pt, 10, engine='sweep')
    assert ctx.apply_edge_cap(10)['applied']
    ctx.components()
    a, b, _, _ = ctx.edges(ctx.stats()['n_edges'])
    np.testing.assert_array_equal(ctx.labels(), union_find_labels(c2.n_reads, a, b))


@pytest.mark.parametrize('engine', ['walk', 'auto'])
def test_zero_division_raises(ctx, engine):
    data, _, _ = host_prepare('zerodiv')
    csr = data.csr()
    with pytest.raises(ZeroDivisionError):
        gpu_run(ctx, csr, engine=engine)


@pytest.mark.parametrize('engine', ENGINES)
def test_zero_qlen2_pair_raises(ctx, engine):
    """Two overlapping reads with qlen2 == 0 (no aln_size == 0 interval, so the sweep may run):
    different_lengths_or_alignments divides by zero (cluster.py:178-183)."""
    off = np.array([0, 1, 2], np.int64)
    chrom = np.zeros(2, np.int32)
    start = np.array([5000, 5010], np.int32)
    end = start + 1000
    aln = np.full(2, 1000, np.int64)
    ctx.set_reads(off, np.zeros(2, np.int32), np.zeros(2, np.int32), chrom, start, end,
                  fold_overlap_threshold(aln, 0.8), 1, iv_data_pos=np.arange(2))
    ctx.reserve_edges(16)
    ctx.build_index()
    with pytest.raises(ZeroDivisionError):
        ctx.run_query(1 - 0.04, 1 - 0.25, pass_table([1.0]), engine=engine)


# ------------------------------------------------------------------ KATs through the device
@pytest.mark.parametrize('engine', ENGINES)
def test_kat_jaccard_on_device(ctx, engine):
    """Each KAT pair becomes two reads on a private coordinate range; the device
    must report exactly the reference's n_i (I) and U for every pair with I > 0."""
    kats = [k for k in fx.kats()['jaccard'] if 'raises' not in k and k['pct'] > 0]
    if engine == 'sweep':      # an aln_size == 0 interval is the walk engine's (exact ZeroDivision replay)
        kats = [k for k in kats if all(x[3] > 0 for x in k['a'] + k['b'])]
    reads = []
    for t, k in enumerate(kats):
        base = 10_000 + t * 10_000
        for lst in (k['a'], k['b']):
            reads.append([(c, s + base, e + base, a) for c, s, e, a in lst])
    # reads are ranked by first start; pairs never overlap across KATs
    off = np.zeros(len(reads) + 1, np.int64)
    off[1:] = np.cumsum([len(r) for r in reads])
    flat = [x for r in reads for x in r]
    chrom = np.array([x[0] for x in flat], np.int32)
    start = np.array([x[1] for x in flat], np.int32)
    end = np.array([x[2] for x in flat], np.int32)
    aln = np.array([x[3] for x in flat], np.int64)
    n = len(reads)
    res = {}
    for pct in sorted({k['pct'] for k in kats}):
        thr = fold_overlap_threshold(aln, pct)
        ctx.set_reads(off, np.full(n, 100, np.int32), np.full(n, 3, np.int32), chrom, start, end, thr,
                      int(chrom.max()) + 1)
        ctx.reserve_edges(4 * n)
        ctx.build_index()
        ctx.query(1.0, 1.0, pass_table([0.0]), engine=engine)
        st = ctx.stats()
        assert st['engine'] == engine
        a, b, I, U = ctx.edges(st['n_edges'])
        for x, y, i, u in zip(a.tolist(), b.tolist(), I.tolist(), U.tolist()):
            res[(pct, min(x, y) // 2)] = (i, u)
    for t, k in enumerate(kats):
        got = res.get((k['pct'], t))
        if k['n_i'] == 0:
            assert got is None or got[0] == 0
        else:
            assert got is not None, (t, k)
            assert got[0] == k['n_i'] and got[0] / got[1] == k['j'], (t, k, got)


# ------------------------------------------------------------------ synthetic configs vs oracle
@pytest.mark.parametrize('n,lmax,seed,dist', [
    (100_000, 8, 7, 'uniform'),       # BASELINE config 2
    (20_000, 64, 13, 'zipf'),         # config 5 shape (skewed 1..64), reduced size
    (50_000, 16, 5, 'uniform'),
])
@pytest.mark.parametrize('engine', ENGINES)
def test_synthetic_vs_oracle(ctx, n, lmax, seed, dist, engine):
    s = synth.generate(n, lmax, seed, dist=dist)
    csr = s.interval_data().csr()
    g = gpu_run(ctx, csr, engine=engine)
    o = O.run_core(oracle_from_csr(csr), use_cap=False)
    compare_with_oracle(g, o, csr.n_reads)


@pytest.mark.parametrize('params', [
    dict(overlap=0.5, cutoffs=(1, 0.5, 0.5), qlen_diff=0.1, nal_diff=0.5),
    dict(overlap=0.0, cutoffs=(0.2,), qlen_diff=0.04, nal_diff=0.25),
    dict(overlap=0.95, cutoffs=(0.3,), qlen_diff=0.0, nal_diff=0.0),
])
@pytest.mark.parametrize('engine', ['walk', 'auto'])
def test_parameter_variants_vs_oracle(ctx, params, engine):
    s = synth.generate(20_000, 8, 23)
    csr = s.interval_data().csr()
    g = gpu_run(ctx, csr, engine=engine, **params)
    # overlap <= 0 (thresholds < 1: matches need not overlap) is the walk engine's
    assert g['stats']['engine'] == ('walk' if engine == 'walk' or params['overlap'] <= 0 else 'sweep')
    o = O.run_core(oracle_from_csr(csr), params['overlap'], params['cutoffs'], params['qlen_diff'],
                   params['nal_diff'], use_cap=False)
    compare_with_oracle(g, o, csr.n_reads)


@pytest.mark.slow
def test_config3_1m_vs_oracle(ctx):
    """BASELINE config 3 (1M reads, 1-16 fillings): full bit-exact comparison, both engines."""
    s = synth.generate(1_000_000, 16, 11)
    csr = s.interval_data().csr()
    o = O.run_core(oracle_from_csr(csr), use_cap=False)
    for engine in ENGINES:
        g = gpu_run(ctx, csr, engine=engine)
        compare_with_oracle(g, o, csr.n_reads)


@pytest.mark.parametrize('engine', ENGINES)
def test_full_sort_index_path_matches_data_order_path(ctx, engine):
    """Index built by the (chrom, start) radix sort == index built from the host's start order."""
    s = synth.generate(40_000, 16, 4)
    csr = s.interval_data().csr()
    g1 = gpu_run(ctx, csr, full_sort=True, engine=engine)
    g2 = gpu_run(ctx, csr, engine=engine)
    np.testing.assert_array_equal(g1['labels'], g2['labels'])
    np.testing.assert_array_equal(g1['fwd'], g2['fwd'])
    assert sorted(zip(g1['a'], g1['b'], g1['I'])) == sorted(zip(g2['a'], g2['b'], g2['I']))
    assert g1['stats']['evaluated_pairs'] == g2['stats']['evaluated_pairs']


@pytest.mark.parametrize('split,mod', [(3, 64), (5, None)])
@pytest.mark.parametrize('engine', ENGINES)
def test_many_chromosomes_vs_oracle(ctx, split, mod, engine):
    """Chromosome counts at the index build's limits: 64 ids (the largest the counting-sort pass
    takes, every chromosome bit in use) and 115 ids (the radix-pass fallback)."""
    import dataclasses
    s = synth.generate(30_000, 16, 37)
    csr = s.interval_data().csr()
    ch = csr.iv_chrom.astype(np.int64) * split + (csr.iv_start.astype(np.int64) // 1000) % split
    if mod:
        ch %= mod
    _, dense = np.unique(ch, return_inverse=True)
    csr = dataclasses.replace(csr, iv_chrom=dense.astype(np.int32), n_chroms=int(dense.max()) + 1)
    assert csr.n_chroms == (mod or 23 * split)
    g = gpu_run(ctx, csr, engine=engine)
    o = O.run_core(oracle_from_csr(csr), use_cap=False)
    compare_with_oracle(g, o, csr.n_reads)


@pytest.mark.parametrize('engine', ENGINES)
@pytest.mark.parametrize('squeeze', [100, 400])
def test_dense_overlaps_vs_oracle(ctx, squeeze, engine):
    """Dense inputs (the 10M-read config's regime): starts squeezed onto 1/squeeze of the genome,
    so walks run to ~350 / ~1400 records per read and reads take several partner partitions."""
    import dataclasses
    s = synth.generate(30_000, 16, 41)
    csr = s.interval_data().csr()
    st = csr.iv_start.astype(np.int64) // squeeze          # monotone: the data order stays start-sorted
    en = st + (csr.iv_end.astype(np.int64) - csr.iv_start)
    csr = dataclasses.replace(csr, iv_start=st.astype(np.int32), iv_end=en.astype(np.int32))
    g = gpu_run(ctx, csr, engine=engine)
    o = O.run_core(oracle_from_csr(csr), use_cap=False)
    compare_with_oracle(g, o, csr.n_reads)


@pytest.mark.parametrize('n_shards', [3])
def test_dense_shards_with_partitioned_launch_vs_oracle(n_shards):
    """Dense input (most reads handed to the partitioned launch) queried as shards of a
    shard-built index (fslr_set_shard), one context per shard: the union of the shards' edges,
    forward degrees and pair counts equals the oracle's."""
    import dataclasses
    s = synth.generate(20_000, 16, 43)
    csr = s.interval_data().csr()
    st0 = csr.iv_start.astype(np.int64) // 400
    en0 = st0 + (csr.iv_end.astype(np.int64) - csr.iv_start)
    csr = dataclasses.replace(csr, iv_start=st0.astype(np.int32), iv_end=en0.astype(np.int32))
    o = O.run_core(oracle_from_csr(csr), use_cap=False)
    thr = fold_overlap_threshold(csr.iv_aln, 0.8)
    pt = pass_table([1, 1, 0.66, 0.66, 0.66, 0.5])
    edges, pairs = [], 0
    fwd = np.zeros(csr.n_reads, np.int64)
    for r in range(n_shards):
        c = _lib.Context(0)
        c.load_csr(csr, thr)
        c.reserve_edges(64 * csr.n_reads)
        c.set_shard(r, n_shards)
        c.build_index()
        c.reserve_deferred(1 << 24)
        c.query_shard(1 - 0.04, 1 - 0.25, pt, r, n_shards)
        st = c.stats()
        pairs += st['evaluated_pairs']
        edges += list(zip(*[x.tolist() for x in c.edges(st['n_edges'])]))
        own = (np.arange(csr.n_reads) // 64) % n_shards == r
        fwd[own] = c.fwd_degree()[own]
        c.close()
    assert pairs == o['stats']['evaluated_pairs']
    assert sorted(edges) == sorted(zip(o['edge_a'].tolist(), o['edge_b'].tolist(), o['edge_I'].tolist(),
                                       o['edge_U'].tolist()))
    np.testing.assert_array_equal(fwd, o['fwd'])


@pytest.mark.parametrize('pass_records,engine', [(None, 'walk'), ('0', 'walk'), ('500', 'walk'), (None, 'sweep')])
def test_one_locus_many_partners_vs_oracle(ctx, monkeypatch, pass_records, engine):
    """1500 reads on one interval: every pair overlaps.  Default: up to 6 partner partitions per
    read; '0': one partition, the hash overflows (witness path); '500': partitions of ~500 partners,
    which overflow within a partition."""
    if pass_records is not None:
        monkeypatch.setenv('FSLR_PASS_RECORDS', pass_records)
    n = 1500
    off = np.arange(n + 1, dtype=np.int64)
    chrom = np.zeros(n, np.int32)
    start = np.full(n, 5000, np.int32) + (np.arange(n) % 7).astype(np.int32)
    start = np.sort(start)
    end = start + 1000
    aln = np.full(n, 1000, np.int64)
    q = np.full(n, 100, np.int32)
    m = np.full(n, 3, np.int32)
    thr = fold_overlap_threshold(aln, 0.8)
    ctx.set_reads(off, q, m, chrom, start, end, thr, 1, iv_data_pos=np.arange(n))
    ctx.reserve_edges(n * n)
    ctx.build_index()
    st = ctx.run_query(1 - 0.04, 1 - 0.25, pass_table([1.0]), engine=engine)
    assert st['engine'] == engine
    ctx.components()
    a, b, I, U = ctx.edges(st['n_edges'])
    g = dict(stats=st, labels=ctx.labels(), fwd=ctx.fwd_degree(), a=a, b=b, I=I, U=U)
    o = O.run_core(O.OracleCSR(off, chrom, start, end, aln, q, m, np.arange(n)), 0.8, (1.0,), 0.04, 0.25,
                   use_cap=False)
    if pass_records is not None:
        assert st['overflow_candidates'] > 0
    compare_with_oracle(g, o, n)


@pytest.mark.parametrize('engine', ENGINES)
def test_rerun_is_deterministic(ctx, engine):
    s = synth.generate(30_000, 16, 2)
    csr = s.interval_data().csr()
    g1 = gpu_run(ctx, csr, engine=engine)
    g2 = gpu_run(ctx, csr, engine=engine)
    np.testing.assert_array_equal(g1['labels'], g2['labels'])
    np.testing.assert_array_equal(g1['fwd'], g2['fwd'])
    assert sorted(zip(g1['a'], g1['b'])) == sorted(zip(g2['a'], g2['b']))


@pytest.mark.parametrize('engine', ENGINES)
def test_vectors_cluster_ids(ctx, engine):
    """Committed reference cluster-id vectors (10k / 20k reads) through the device path."""
    for vec in ('v10k_l8_s7', 'v20k_l16_s11'):
        z = np.load(os.path.join(fx.GOLDEN, 'vectors', f'{vec}.npz'))
        n, lmax, seed = (int(x) for x in z['params'])
        s = synth.generate(n, lmax, seed)
        data = s.interval_data()
        csr = data.csr()
        g = gpu_run(ctx, csr, engine=engine)
        lab = g['labels']
        sizes = np.bincount(lab, minlength=csr.n_reads)
        roots = np.flatnonzero(sizes >= 2)
        rid = np.full(csr.n_reads, -1)
        rid[roots] = np.arange(roots.size)
        comp_rank = np.where(sizes[lab] >= 2, rid[lab], -1)
        comp = np.full(n, -1, np.int32)
        comp[csr.read_qcode] = comp_rank       # qcode == read number for the generator path
        fwd = np.zeros(n, np.int32)
        fwd[csr.read_qcode] = g['fwd']
        np.testing.assert_array_equal(comp, z['comp'])
        np.testing.assert_array_equal(fwd, z['fwd'])


# ------------------------------------------------------------------ length gate at ratio boundaries
def _boundary_pool(cut, top, rng):
    """Values v and partners just inside / outside fl(min/max) >= cut for several magnitudes."""
    pool = {1, 2, 3, top}
    for v in (1, 2, 7, 25, 100, 1000, 12345, 1 << 20, top):
        pool.add(v)
        if cut > 0:
            for x in (int(np.floor(cut * v)), int(np.ceil(v / cut)) if cut <= 1 else v):
                for d in (-1, 0, 1):
                    if 1 <= x + d <= top:
                        pool.add(x + d)
    pool = np.array(sorted(pool), np.int64)
    return pool[rng.integers(0, pool.size, 400)]


@pytest.mark.parametrize('engine', ENGINES)
@pytest.mark.parametrize('qlen_diff,nal_diff', [(0.04, 0.25), (0.0, 0.0), (1.0, 1.0), (1.5, -0.5), (-0.5, 1.5),
                                                (0.34, 0.999999), (1e-12, 0.5)])
def test_length_gate_boundaries_vs_oracle(ctx, monkeypatch, qlen_diff, nal_diff, engine):
    """400 reads with one identical interval each (every pair overlaps, so every pair is evaluated
    and the first reads overflow the per-read partner hash): qlen2 / n_alignments drawn around the
    exact ratio boundaries of cluster.py:178-183; one read each with qlen2 == 0 and nal == 0."""
    monkeypatch.setenv('FSLR_PASS_RECORDS', '0')      # one partner partition: the hash overflows
    rng = np.random.default_rng(int(1000 * (qlen_diff + 2 * nal_diff)) & 0xFFFF)
    n = 400
    q = _boundary_pool(1 - qlen_diff, (1 << 31) - 1, rng)
    m = _boundary_pool(1 - nal_diff, (1 << 24) - 1, rng)
    q[17] = 0
    m[211] = 0
    off = np.arange(n + 1, dtype=np.int64)
    chrom = np.zeros(n, np.int32)
    start = np.full(n, 5000, np.int32)
    end = np.full(n, 6000, np.int32)
    aln = np.full(n, 1000, np.int64)
    thr = fold_overlap_threshold(aln, 0.8)
    ctx.set_reads(off, q.astype(np.int32), m.astype(np.int32), chrom, start, end, thr, 1)
    ctx.reserve_edges(n * n)
    ctx.build_index()
    st = ctx.run_query(1 - qlen_diff, 1 - nal_diff, pass_table([1.0]), engine=engine)
    ctx.components()
    a, b, I, U = ctx.edges(st['n_edges'])
    g = dict(stats=st, labels=ctx.labels(), fwd=ctx.fwd_degree(), a=a, b=b, I=I, U=U)
    o = O.run_core(O.OracleCSR(off, chrom, start, end, aln, q, m, np.arange(n)), 0.8, (1.0,), qlen_diff, nal_diff,
                   use_cap=False)
    assert engine == 'sweep' or st['overflow_candidates'] > 0
    compare_with_oracle(g, o, n)


@pytest.mark.parametrize('n_shards', [2, 3, 8])
def test_query_shards_partition_the_pairs(ctx, n_shards):
    """fslr_query_shard over all shards evaluates exactly the pairs and edges of one full query."""
    s = synth.generate(25_000, 16, 19)
    csr = s.interval_data().csr()
    o = O.run_core(oracle_from_csr(csr), use_cap=False)
    thr = fold_overlap_threshold(csr.iv_aln, 0.8)
    ctx.load_csr(csr, thr)
    ctx.reserve_edges(12 * csr.n_reads)
    ctx.build_index()
    pt = pass_table([1, 1, 0.66, 0.66, 0.66, 0.5])
    edges, pairs = [], 0
    fwd = np.zeros(csr.n_reads, np.int64)
    for r in range(n_shards):
        ctx.query_shard(1 - 0.04, 1 - 0.25, pt, r, n_shards)
        st = ctx.stats()
        pairs += st['evaluated_pairs']
        a, b, I, U = ctx.edges(st['n_edges'])
        assert np.all((a // 64) % n_shards == r)
        edges += list(zip(a.tolist(), b.tolist(), I.tolist(), U.tolist()))
        f = ctx.fwd_degree()
        own = (np.arange(csr.n_reads) // 64) % n_shards == r
        fwd[own] = f[own]
    assert pairs == o['stats']['evaluated_pairs']
    oe = sorted(zip(o['edge_a'].tolist(), o['edge_b'].tolist(), o['edge_I'].tolist(), o['edge_U'].tolist()))
    assert sorted(edges) == oe
    np.testing.assert_array_equal(fwd, o['fwd'])


@pytest.mark.parametrize('n_shards', [1, 3])
def test_work_queue_read_assignment_vs_oracle(ctx, monkeypatch, n_shards):
    """The pair kernel's work-queue read assignment (used when every wave holds >= 64 reads, e.g.
    1M reads on one GPU) forced on at 60k reads: same edges, degrees and pair counts as the oracle."""
    monkeypatch.setenv('FSLR_DYNAMIC_MIN_READS', '0')
    s = synth.generate(60_000, 16, 31)
    csr = s.interval_data().csr()
    o = O.run_core(oracle_from_csr(csr), use_cap=False)
    if n_shards == 1:
        compare_with_oracle(gpu_run(ctx, csr), o, csr.n_reads)
        return
    thr = fold_overlap_threshold(csr.iv_aln, 0.8)
    ctx.load_csr(csr, thr)
    ctx.reserve_edges(12 * csr.n_reads)
    ctx.build_index()
    pt = pass_table([1, 1, 0.66, 0.66, 0.66, 0.5])
    edges, pairs = [], 0
    fwd = np.zeros(csr.n_reads, np.int64)
    for r in range(n_shards):
        ctx.query_shard(1 - 0.04, 1 - 0.25, pt, r, n_shards)
        st = ctx.stats()
        pairs += st['evaluated_pairs']
        edges += list(zip(*[x.tolist() for x in ctx.edges(st['n_edges'])]))
        own = (np.arange(csr.n_reads) // 64) % n_shards == r
        fwd[own] = ctx.fwd_degree()[own]
    assert pairs == o['stats']['evaluated_pairs']
    assert sorted(edges) == sorted(zip(o['edge_a'].tolist(), o['edge_b'].tolist(), o['edge_I'].tolist(),
                                       o['edge_U'].tolist()))
    np.testing.assert_array_equal(fwd, o['fwd'])


def test_shard_built_index_matches_full_index():
    """fslr_set_shard: an index whose query-side data covers one shard gives that shard exactly
    the edges of a fully built index; the full-range query is refused on it."""
    s = synth.generate(25_000, 16, 29)
    csr = s.interval_data().csr()
    thr = fold_overlap_threshold(csr.iv_aln, 0.8)
    pt = pass_table([1, 1, 0.66, 0.66, 0.66, 0.5])
    full = _lib.Context(0)
    full.load_csr(csr, thr)
    full.reserve_edges(12 * csr.n_reads)
    full.build_index()
    for r in range(4):
        c = _lib.Context(0)
        c.load_csr(csr, thr)
        c.reserve_edges(12 * csr.n_reads)
        c.set_shard(r, 4)
        c.build_index()
        c.query_shard(1 - 0.04, 1 - 0.25, pt, r, 4)
        st = c.stats()
        full.query_shard(1 - 0.04, 1 - 0.25, pt, r, 4)
        sf = full.stats()
        assert st['evaluated_pairs'] == sf['evaluated_pairs']
        assert sorted(zip(*[x.tolist() for x in c.edges(st['n_edges'])])) == \
            sorted(zip(*[x.tolist() for x in full.edges(sf['n_edges'])]))
        with pytest.raises(_lib.FslrError):
            c.query(1 - 0.04, 1 - 0.25, pt)
        c.close()
    full.close()


def _multi_inputs(name):
    from fslr_amd.prep import fold_overlap_threshold, pass_table
    data, _, kw = host_prepare(name)
    csr = data.csr()
    cut = [float(x) for x in kw['jaccard_cutoffs'].split(',')]
    return csr, fold_overlap_threshold(csr.iv_aln, kw['overlap']), kw, pass_table(cut)


def test_rank_pool_is_reused_across_queries():
    """The CLI's persistent ranks (fslr_amd.multi.RankPool): two queries on the same children (same
    PIDs), each equal to the single-GPU oracle's graph (edges, forward degrees)."""
    from fslr_amd import multi
    pool = multi.pool(2)
    pids = sorted(p.pid for p in pool.procs.values())
    for name in ('capbind_1500', 'mixed_2k_l8'):
        csr, thr, kw, pt = _multi_inputs(name)
        r = multi.query(csr, thr, 1 - kw['qlen_diff'], 1 - kw['n_alignment_diff'], pt, 10, 2)
        o = O.run_core(oracle_from_csr(csr), kw['overlap'], [float(x) for x in kw['jaccard_cutoffs'].split(',')],
                       kw['qlen_diff'], kw['n_alignment_diff'], 10, use_cap=True)
        a, b, I, U = r['edges']
        assert sorted(zip(a.tolist(), b.tolist(), I.tolist(), U.tolist())) == sorted(
            zip(o['edge_a'].tolist(), o['edge_b'].tolist(), o['edge_I'].tolist(), o['edge_U'].tolist()))
        np.testing.assert_array_equal(r['fwd'], o['fwd'])
        assert multi.pool(2) is pool and sorted(p.pid for p in pool.procs.values()) == pids


def test_rank_pool_child_rank0_raises_zero_division(monkeypatch):
    """Rank 0 as a child process (the caller's HIP runtime already up without torch's): its
    ZeroDivisionError reaches the caller with its type, and the pool stays usable."""
    from fslr_amd import multi
    monkeypatch.setattr(multi, '_rank0_in_process', lambda: False)
    pool = multi.RankPool(2)
    try:
        assert 0 in pool.procs
        import dataclasses
        csr, thr, kw, pt = _multi_inputs('cfg1_1k_x3')
        q2 = csr.read_qlen2.copy()
        q2[::3] = 0                                  # pairs of two qlen2-0 reads raise (cluster.py:178-183)
        csr = dataclasses.replace(csr, read_qlen2=q2)
        assert multi.sweep_applies(csr, thr)
        with pytest.raises(ZeroDivisionError):
            O.run_core(oracle_from_csr(csr), use_cap=True)
        with pytest.raises(ZeroDivisionError):
            pool.query(csr, thr, 1 - kw['qlen_diff'], 1 - kw['n_alignment_diff'], pt, 10)
        assert pool.alive()
        csr, thr, kw, pt = _multi_inputs('cfg1_1k_x3')
        r = pool.query(csr, thr, 1 - kw['qlen_diff'], 1 - kw['n_alignment_diff'], pt, 10)
        o = O.run_core(oracle_from_csr(csr), use_cap=True)
        assert sorted(zip(r['edges'][0].tolist(), r['edges'][1].tolist())) == sorted(
            zip(o['edge_a'].tolist(), o['edge_b'].tolist()))
    finally:
        pool.close()
