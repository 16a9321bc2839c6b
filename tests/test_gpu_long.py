"""GPU parity for reads of more than FSLR_MAX_L (64) intervals (fslr_long_evaluate).

The reference has no per-read interval limit (overall_jaccard_similarity, cluster.py:140-170); the
device uploads such reads as <= 64-interval chunks and decides their pairs with the first-fit over the
whole lists.  Bar: the oracle's edges (a, b, I, U), forward degrees and components, bit for bit.
"""
import numpy as np
import pytest

from fslr_amd import cluster, synth
from oracle import oracle as O

from test_gpu_parity import oracle_from_csr

pytestmark = pytest.mark.gpu

CUTS = [1, 1, 0.66, 0.66, 0.66, 0.5]


@pytest.mark.parametrize('n,lmin,lmax,seed,overlap,cuts', [
    (3000, 1, 150, 3, 0.8, CUTS),     # long reads among short ones (short-long, long-long, short-short pairs)
    (1500, 60, 300, 4, 0.8, CUTS),    # mostly long reads, up to 300 intervals
    (800, 65, 65, 5, 0.8, CUTS),      # every read exactly 65 intervals (one extra chunk of one interval)
    (3000, 1, 150, 6, 0.05, [0.3]),   # loose overlap: many matching interval pairs, first-fit conflicts
])
def test_long_reads_vs_oracle(n, lmin, lmax, seed, overlap, cuts):
    s = synth.generate(n, lmax, seed, lmin=lmin)
    data = s.interval_data()
    csr = data.csr()
    assert np.diff(csr.read_off).max() > 64
    idx = cluster.build_interval_trees(data)
    assert idx.long is not None
    match_df, G = cluster.query_interval_trees(idx, data, overlap, cuts, 10, 0.04, 0.25)
    a, b = G.edges_ab
    I_U = match_df['jaccard_similarity'].to_numpy()
    o = O.run_core(oracle_from_csr(csr), overlap=overlap, cutoffs=cuts, use_cap=False)
    assert G.stats['engine'] == 'sweep+long'
    assert G.stats['long_reads'] > 0
    # edges with I, U: match_df holds I/U; the oracle's (a, b, I, U) give the same floats
    oe = sorted(zip(o['edge_a'].tolist(), o['edge_b'].tolist()))
    ge = sorted(zip(a.tolist(), b.tolist()))
    assert ge == oe
    ok = dict(zip(zip(o['edge_a'].tolist(), o['edge_b'].tolist()), (o['edge_I'] / o['edge_U']).tolist()))
    assert [ok[(x, y)] for x, y in zip(a.tolist(), b.tolist())] == I_U.tolist()
    np.testing.assert_array_equal(G.fwd, o['fwd'])
    assert G.stats['max_fwd'] == o['stats']['max_fwd']
    # the uncapped oracle equals the reference loop here (the cap does not bind)
    oc = O.run_core(oracle_from_csr(csr), overlap=overlap, cutoffs=cuts, use_cap=True)
    assert sorted(zip(oc['edge_a'].tolist(), oc['edge_b'].tolist())) == oe
    np.testing.assert_array_equal(G.component_id, o['comp'])
    assert G.stats['long_pair_edges'] > 0


def _capped_equal(G, match_df, o):
    """The capped graph against the reference loop: edges as (former, partner) with I/U, forward
    degrees (edges formed in each read's own loop), components."""
    a, b = G.edges_ab
    want = sorted(zip(o['edge_a'].tolist(), o['edge_b'].tolist(), (o['edge_I'] / o['edge_U']).tolist()))
    got = sorted(zip(a.tolist(), b.tolist(), match_df['jaccard_similarity'].tolist()))
    assert got == want
    np.testing.assert_array_equal(G.fwd, o['fwd'])
    np.testing.assert_array_equal(G.component_id, o['comp'])


def _squeezed_long(n, lmin, lmax, seed, squeeze, ccap):
    """Long reads in dense events on a squeezed genome: the cap binds with long reads in the loops."""
    import dataclasses
    s = synth.generate(n, lmax, seed, lmin=lmin, cluster_cap=ccap, size_p=0.02)
    data = s.interval_data()
    st = data.start.astype(np.int64) // squeeze
    en = st + (data.end.astype(np.int64) - data.start)
    return dataclasses.replace(data, start=st.astype(data.start.dtype), end=en.astype(data.end.dtype), _csr=None)


@pytest.mark.parametrize('overlap,cuts', [(0.8, CUTS), (0.0, [0.2]), (-0.5, [0.3])])
@pytest.mark.parametrize('thr', [10, 3])
def test_long_reads_dense_locus_capped_vs_oracle(thr, overlap, cuts):
    """One dense locus (every read overlaps every other): forward degrees far above the cap, so the
    reference's loops break; the replay in the real-read space (fslr_cap_replay_pairs) gives its graph.
    overlap <= 0 takes the general pair evaluator (fslr_long_pairs) for E*."""
    s = synth.generate(400, 80, 7, lmin=70, cluster_cap=400, size_p=0.001)
    data = s.interval_data()
    csr = data.csr()
    idx = cluster.build_interval_trees(data)
    match_df, G = cluster.query_interval_trees(idx, data, overlap, cuts, thr, 0.04, 0.25)
    o = O.run_core(oracle_from_csr(csr), overlap=overlap, cutoffs=cuts, edge_threshold=thr, use_cap=True)
    assert G.stats['engine'] == ('sweep+long' if overlap > 0 else 'pairs')
    assert G.stats['cap']['applied'] == 1 and G.stats['max_fwd'] > thr
    _capped_equal(G, match_df, o)


@pytest.mark.parametrize('overlap,cuts,thr', [(0.8, CUTS, 10), (0.8, CUTS, 2), (0.0, [0.2], 10), (0.05, [0.3], 4)])
def test_long_reads_squeezed_capped_vs_oracle(overlap, cuts, thr):
    """Short and long reads (1..150 fillings) in events of up to 60 reads: chains of pairs left unseen
    by capped loops across long and short reads."""
    data = _squeezed_long(2500, 1, 150, 21, 200, 60)
    csr = data.csr()
    assert np.diff(csr.read_off).max() > 64
    idx = cluster.build_interval_trees(data)
    match_df, G = cluster.query_interval_trees(idx, data, overlap, cuts, thr, 0.04, 0.25)
    o = O.run_core(oracle_from_csr(csr), overlap=overlap, cutoffs=cuts, edge_threshold=thr, use_cap=True)
    assert G.stats['cap']['applied'] == 1
    _capped_equal(G, match_df, o)


@pytest.mark.parametrize('overlap', [0.0, -1.0, 0.8])
def test_long_reads_general_path_vs_oracle(overlap):
    """The general evaluator (overlap <= 0: matches need not overlap) on sparse long reads; the cap
    binds for a few reads at overlap 0."""
    s = synth.generate(1500, 120, 8, lmin=1)
    data = s.interval_data()
    csr = data.csr()
    idx = cluster.build_interval_trees(data)
    o = O.run_core(oracle_from_csr(csr), overlap=overlap, cutoffs=[0.5], use_cap=True)
    match_df, G = cluster.query_interval_trees(idx, data, overlap, [0.5], 10, 0.04, 0.25)
    if overlap <= 0:
        assert G.stats['engine'] == 'pairs'
    _capped_equal(G, match_df, o)


def test_long_reads_zero_aln_raises_like_the_reference():
    s = synth.generate(600, 100, 9, lmin=40)
    data = s.interval_data()
    import dataclasses
    aln = data.aln_size.copy()
    aln[::37] = 0
    data = dataclasses.replace(data, aln_size=aln, _csr=None)
    csr = data.csr()
    with pytest.raises(ZeroDivisionError):
        O.run_core(oracle_from_csr(csr), use_cap=True)
    idx = cluster.build_interval_trees(data)
    with pytest.raises(ZeroDivisionError):
        cluster.query_interval_trees(idx, data, 0.8, CUTS, 10, 0.04, 0.25)
