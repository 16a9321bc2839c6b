"""BASELINE configs 4 and 5 on the GPU (the largest inputs of the parity suite).

* cfg4: 1M reads split into 8 query shards (the multi-GPU partition, fslr_set_shard /
  fslr_query_shard, one context per shard on one GPU), per-shard components merged by
  union of the shards' label vectors (what DeviceShardMerge does after its RCCL
  all_gather): identical labels, edges and pair counts to one full context, and the
  CPU oracle's pair / edge counts.
* cfg5: 10M reads, 1-64 fillings (truncated Zipf 1.5): the edge cap binds (forward
  degrees up to 28); the capped graph of the full run, restricted to the loops of query
  reads [0, 50000), equals the oracle's reference loop over those reads
  (tests/golden/cfg5/sample50k_capped.npz, made by tests/golden/make_cfg5_sample.py), and the
  whole capped graph (every edge with I, U, the forward degrees and the labels of all 10M reads)
  has the digests of the oracle's full run (tests/golden/cfg5/full_capped.json).
* cfg4 input through the product's chromosome split: W = 8 ranks on one GPU, each rank's capped
  graph and labels against the oracle's full 1M-read digests (tests/golden/cfg5/cfg4_1m.json).
"""
import json
import os
import sys

import numpy as np
import pytest

from fslr_amd import _lib, synth
from fslr_amd.prep import fold_overlap_threshold, pass_table
from oracle import oracle as O

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), 'golden')
sys.path.insert(0, GOLDEN)
CUTS = [1, 1, 0.66, 0.66, 0.66, 0.5]


@pytest.mark.slow
def test_config4_1m_eight_shards_merge_to_the_full_run():
    s = synth.generate(1_000_000, 16, 11)
    csr = s.interval_data().csr()
    thr = fold_overlap_threshold(csr.iv_aln, 0.8)
    pt = pass_table(CUTS)
    full = _lib.Context(0)
    full.load_csr(csr, thr)
    full.reserve_edges(12 * csr.n_reads)
    full.build_index()
    fst = full.run_query(1 - 0.04, 1 - 0.25, pt, engine='walk')
    assert full.apply_edge_cap(10)['applied'] == 0          # cfg3/4: the cap does not bind
    full.components()
    want_labels = full.labels()
    want_edges = sorted(zip(*[x.tolist() for x in full.edges(fst['n_edges'])]))
    want_fwd = full.fwd_degree()
    # the position-sweep engine on the same context: the same edges, degrees and components
    sst = full.run_query(1 - 0.04, 1 - 0.25, pt, engine='sweep')
    assert sst['engine'] == 'sweep' and sst['n_edges'] == fst['n_edges']
    assert sorted(zip(*[x.tolist() for x in full.edges(sst['n_edges'])])) == want_edges
    np.testing.assert_array_equal(full.fwd_degree(), want_fwd)
    full.components()
    np.testing.assert_array_equal(full.labels(), want_labels)
    W = 8
    labels, edges, pairs, jacc = [], [], 0, 0
    for r in range(W):
        c = _lib.Context(0)
        c.load_csr(csr, thr)
        c.reserve_edges(4 * csr.n_reads)
        c.set_shard(r, W)
        c.build_index()
        c.query_shard(1 - 0.04, 1 - 0.25, pt, r, W)
        st = c.stats()
        pairs += st['evaluated_pairs']
        jacc += st['jaccard_evals']
        a, b, I, U = c.edges(st['n_edges'])
        assert np.all((a // 64) % W == r)
        edges += list(zip(a.tolist(), b.tolist(), I.tolist(), U.tolist()))
        c.components()
        labels.append(c.labels())
        c.close()
    assert pairs == fst['evaluated_pairs'] and jacc == fst['jaccard_evals']
    assert sorted(edges) == want_edges
    # the merge: union (k, label_g[k]) over every shard g, on one context's forest
    m = _lib.Context(0)
    m.load_csr(csr, thr)
    m.components()                       # no query: every read its own root
    m.union_pairs(None, np.concatenate(labels), W * csr.n_reads, on_device=False)
    m.finalize_labels()
    np.testing.assert_array_equal(m.labels(), want_labels)
    m.close()
    full.close()
    # the CPU restatement's counts (all cores, E*)
    cnt = np.diff(csr.read_off)
    oc = O.OracleCSR(csr.read_off, csr.iv_chrom, csr.iv_start, csr.iv_end, csr.iv_aln,
                     np.repeat(csr.read_qlen2, cnt), np.repeat(csr.read_nal, cnt), csr.data_pos)
    oct_ = O.count_threads(oc, nthreads=min(16, os.cpu_count() or 1))
    assert (oct_['evaluated_pairs'], oct_['jaccard_evals'], oct_['n_edges']) == (pairs, jacc, len(edges))


@pytest.mark.slow
def test_config5_10m_capped_vs_oracle():
    with open(os.path.join(GOLDEN, 'cfg5', 'sample50k_capped.json')) as fh:
        meta = json.load(fh)
    z = np.load(os.path.join(GOLDEN, 'cfg5', 'sample50k_capped.npz'))
    s = synth.generate(meta['reads'], meta['lmax'], meta['seed'], dist=meta['dist'])
    csr = s.interval_data().csr()
    del s
    assert csr.n_intervals == meta['n_intervals']
    S = meta['sample']
    ctx = _lib.Context(0)
    ctx.load_csr(csr, fold_overlap_threshold(csr.iv_aln, 0.8))
    ctx.reserve_edges(12 * csr.n_reads)
    ctx.reserve_deferred(64 << 20)
    ctx.build_index()
    want = sorted(zip(z['a'].tolist(), z['b'].tolist(), z['I'].tolist(), z['U'].tolist()))
    from make_cfg5_full import digests
    with open(os.path.join(GOLDEN, 'cfg5', 'full_capped.json')) as fh:
        ref = json.load(fh)
    full = {k: ref[k] for k in ('edges_sha256', 'fwd_sha256', 'labels_sha256', 'n_edges', 'max_fwd')}
    labels = {}
    for engine in ('sweep', 'walk'):
        st = ctx.run_query(1 - 0.04, 1 - 0.25, pass_table(CUTS), engine=engine)
        assert st['engine'] == engine
        assert st['max_fwd'] > 10                               # the cap binds at this density
        cap = ctx.apply_edge_cap(10)
        assert cap['applied'] == 1 and cap['dropped'] > 0
        ne = ctx.stats()['n_edges']
        a, b, I, U = ctx.edges(ne)
        own = a < S                                              # edges formed in the loops of reads < S
        got = sorted(zip(a[own].tolist(), b[own].tolist(), I[own].tolist(), U[own].tolist()))
        assert len(got) == len(want) == meta['n_edges']
        assert got == want
        fwd = ctx.fwd_degree()
        np.testing.assert_array_equal(fwd[:S], z['fwd'])
        ctx.components()
        labels[engine] = lab = ctx.labels()
        assert lab.shape == (csr.n_reads,) and np.all(lab <= np.arange(csr.n_reads))
        d = digests(a, b, I, U, fwd, lab)
        assert {k: d[k] for k in full} == full, engine           # the whole 10M-read graph
    np.testing.assert_array_equal(labels['sweep'], labels['walk'])
    ctx.close()


@pytest.mark.slow
@pytest.mark.parametrize('thr', [10, 3])
def test_config4_1m_product_split_w8_vs_oracle(thr):
    """The product's chromosome split (fslr_sweep_partition -> exchange -> fslr_sweep_evaluate on
    each of W = 8 contexts; with a binding cap also the cap exchange and replay of
    dist.SweepShard's capped path) on the 1M-read input: every rank's graph and labels have the
    oracle's digests (thr 10: the cap does not bind, E*; thr 3: it binds)."""
    from make_cfg5_full import digests
    from test_dist import _sweep_shards_threads, _sweep_split_on_device, _union_view
    with open(os.path.join(GOLDEN, 'cfg5', 'cfg4_1m.json')) as fh:
        ref = json.load(fh)
    csr = synth.generate(ref['reads'], ref['lmax'], ref['seed']).interval_data().csr()
    assert csr.n_intervals == ref['n_intervals']
    thr_iv, pt = fold_overlap_threshold(csr.iv_aln, 0.8), pass_table(CUTS)
    key = 'capped3' if thr == 3 else 'estar'
    want = {k: ref[key][k] for k in ('edges_sha256', 'fwd_sha256', 'labels_sha256', 'n_edges', 'max_fwd')}
    if thr == 3:
        ctxs, infos = _sweep_shards_threads(csr, thr_iv, pt, 8, thr)
        assert all(i['capped'] and i['cap']['capped'] > 0 for i in infos)
        a, b, I, U, fwd = _union_view(ctxs)
        views = [digests(a, b, I, U, fwd, c.labels()) for c in ctxs]
    else:
        ctxs, _ = _sweep_split_on_device(csr, thr_iv, pt, 8, thr)
        parts = [c.edges(c.stats()['n_edges']) for c in ctxs]      # each destination's edges
        a, b, I, U = (np.concatenate([p[k] for p in parts]) for k in range(4))
        fwd = np.sum([c.fwd_degree().astype(np.int64) for c in ctxs], axis=0)
        views = [digests(a, b, I, U, fwd, c.labels()) for c in ctxs]
    try:
        for d in views:
            assert {k: d[k] for k in want} == want
    finally:
        for c in ctxs:
            c.close()


@pytest.mark.slow
def test_config5_10m_product_split_w8_capped_vs_oracle():
    """North star's config 5 (10M reads x 1-64 Zipf, the cap binding) through the product's
    dist.SweepShard on W = 8 ranks (threads of this process, one context each, in-process
    collectives): partition, entry exchange, evaluation, then the sharded cap replay (E* rows
    gathered, the candidates' hit components assigned to ranks, each rank replaying its own) — the
    union of the ranks' capped graphs (edges with I, U; edges per loop) and every rank's labels have
    the digests of the oracle's full run (tests/golden/cfg5/full_capped.json)."""
    from make_cfg5_full import digests
    from test_dist import _sweep_shards_threads, _union_view
    with open(os.path.join(GOLDEN, 'cfg5', 'sample50k_capped.json')) as fh:
        meta = json.load(fh)
    with open(os.path.join(GOLDEN, 'cfg5', 'full_capped.json')) as fh:
        ref = json.load(fh)
    want = {k: ref[k] for k in ('edges_sha256', 'fwd_sha256', 'labels_sha256', 'n_edges', 'max_fwd')}
    s = synth.generate(meta['reads'], meta['lmax'], meta['seed'], dist=meta['dist'])
    csr = s.interval_data().csr()
    del s
    assert csr.n_intervals == meta['n_intervals']
    ctxs, infos = _sweep_shards_threads(csr, fold_overlap_threshold(csr.iv_aln, 0.8), pass_table(CUTS), 8, 10)
    try:
        cap = infos[0]['cap']
        assert cap['applied'] == 1 and cap['dropped'] > 0
        a, b, I, U, fwd = _union_view(ctxs)
        for c in ctxs:
            d = digests(a, b, I, U, fwd, c.labels())
            assert {k: d[k] for k in want} == want
    finally:
        for c in ctxs:
            c.close()
