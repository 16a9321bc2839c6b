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


def test_long_reads_cap_binding_is_refused():
    # one dense locus: every read overlaps every other, so forward degrees exceed the cap
    s = synth.generate(400, 80, 7, lmin=70, cluster_cap=400, size_p=0.001)
    data = s.interval_data()
    idx = cluster.build_interval_trees(data)
    with pytest.raises(NotImplementedError):
        cluster.query_interval_trees(idx, data, 0.8, CUTS, 10, 0.04, 0.25)
