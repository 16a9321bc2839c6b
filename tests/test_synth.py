"""The columnar generator path equals the DataFrame host path (CPU)."""
import numpy as np
import pytest

from fslr_amd import cluster, synth


@pytest.mark.parametrize('n,lmax,seed,dist', [(500, 8, 7, 'uniform'), (300, 64, 13, 'zipf'), (400, 16, 3, 'uniform')])
def test_interval_data_matches_dataframe_path(n, lmax, seed, dist):
    s = synth.generate(n, lmax, seed, dist=dist)
    df = s.to_dataframe()
    bed, lens, mask, _ = cluster.rename_chromosomes(df, dict(s.chrom_lengths), {'subtelomere'})
    d1 = cluster.prepare_data(cluster.keep_fillings(bed), mask, lens)
    d2 = s.interval_data()
    for f in ('chrom', 'start', 'end', 'aln_size', 'n_alignments', 'qlen2', 'middle', 'index'):
        np.testing.assert_array_equal(getattr(d1, f), getattr(d2, f), err_msg=f)
    assert list(d1.qnames[d1.qcode]) == list(d2.qnames[d2.qcode])
    c1, c2 = d1.csr(), d2.csr()
    for f in ('read_off', 'read_qlen2', 'read_nal', 'iv_chrom', 'iv_start', 'iv_end', 'iv_aln'):
        np.testing.assert_array_equal(getattr(c1, f), getattr(c2, f), err_msg=f)
    assert list(d1.qnames[c1.read_qcode]) == list(d2.qnames[c2.read_qcode])


def test_generator_properties():
    s = synth.generate(2000, 16, 11)
    fill = s.aln_size != 20
    st = s.rstart[fill]
    assert np.unique(st).size == st.size            # globally distinct filling starts
    assert s.n_alignments.min() >= 3 and s.n_alignments.max() <= 18
