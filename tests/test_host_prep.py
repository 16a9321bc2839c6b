"""Host stages of the product (vectorised) vs the reference's own intermediates (CPU)."""
import math

import numpy as np
import pytest

import fixtures as fx
from host_pipeline import host_prepare
from fslr_amd import prep
from fslr_amd.prep import fold_overlap_threshold, pass_table
from oracle import oracle as O

STAGE_FIXTURES = [f for f in fx.FIXTURES if fx.stage(f) is not None]


@pytest.mark.parametrize('name', STAGE_FIXTURES)
def test_prepare_data_order_matches_reference(name):
    """keep_fillings + prepare_data (+ mask): same list, same order (ties included)."""
    data, _, _ = host_prepare(name)
    mine = [[data.qnames[c], int(s), int(e)] for c, s, e in zip(data.qcode, data.start, data.end)]
    assert mine == fx.stage(name)['data_order']


@pytest.mark.parametrize('name', STAGE_FIXTURES)
def test_csr_matches_oracle_restatement(name):
    data, _, kw = host_prepare(name)
    csr = data.csr()
    from fslr_amd import bam_header
    ocsr, _ = O.restate_prep(fx.input_bed(name), bam_header.get_chromosome_lengths(fx.input_bam(name)),
                             kw['cluster_mask'], kw['filter_false'])
    assert list(data.qnames[csr.read_qcode]) == list(ocsr.qnames)
    np.testing.assert_array_equal(csr.read_off, ocsr.read_off)
    np.testing.assert_array_equal(csr.iv_start, ocsr.start)
    np.testing.assert_array_equal(csr.iv_end, ocsr.end)
    np.testing.assert_array_equal(csr.iv_aln, ocsr.aln)
    np.testing.assert_array_equal(csr.read_qlen2, ocsr.qlen2[ocsr.read_off[:-1]])
    np.testing.assert_array_equal(csr.read_nal, ocsr.nal[ocsr.read_off[:-1]])
    # chromosome equality structure preserved
    a = csr.iv_chrom
    b = ocsr.chrom
    assert len(set(zip(a.tolist(), b.tolist()))) == len(set(a.tolist())) == len(set(b.tolist()))


def test_fold_threshold_matches_kat():
    for k in fx.kats()['overlap']:
        t = fold_overlap_threshold([k['a1'], k['a2']], k['pct'])
        ok = all((o >= x) if x >= 0 else (o <= ~x) for o, x in ((k['o'], int(t[0])), (k['o'], int(t[1]))))
        assert ok == k['ok'], k


@pytest.mark.parametrize('p', [0.8, 0.66, 0.5, 0.3333333333333333, 0.1, 1.0, 1.25, 0.0, -0.0, -0.5, 1e-9,
                               0.7999999999999999, float('nan'), float('inf'), -float('inf')])
def test_fold_threshold_exhaustive(p):
    """o / a >= p (Python floats) == integer fold, over every small (o, a) incl. a < 0, a == 0."""
    alns = list(range(-40, 41)) + [4999, 5000, 5001, 123457]
    t = fold_overlap_threshold(alns, p)
    for a, x in zip(alns, t.tolist()):
        for o in list(range(0, 130)) + [4000, 3999, 4001, 98765, 98766, 98764]:
            if a == 0:
                assert x == prep.FSLR_THR_ZERO_ALN
                continue
            want = (o / a) >= p
            got = (o >= x) if x >= 0 else (o <= ~x)
            assert got == want, (o, a, p, x)


def test_pass_table_matches_kat():
    for k in fx.kats()['cutoff']:
        tab = pass_table(k['cutoffs']).reshape(64, 128)
        for I, row in enumerate(k['pass_table'], start=1):
            assert list(tab[I - 1, I - 1:]) == row


def test_pass_table_empty_raises():
    with pytest.raises(ValueError):
        pass_table([])


def test_pandas_sort_equivalence_on_ties():
    """data_order == DataFrame.sort_values('start') on tie-heavy columns."""
    import pandas as pd
    rng = np.random.default_rng(3)
    for n in (10, 100, 1000, 50_000):
        s = rng.integers(0, max(2, n // 7), size=n)
        df = pd.DataFrame({'start': s})
        np.testing.assert_array_equal(df.sort_values('start').index.to_numpy(), prep.data_order(s))


def test_interval_data_from_reference_items_round_trips():
    """build_interval_trees / query_interval_trees accept the reference's prepare_data output (a
    list of IntervalItem): its columns, ranks and CSR equal those of the columnar data."""
    from fslr_amd import synth
    from fslr_amd.prep import IntervalData
    data = synth.generate(3000, 8, 5).interval_data()
    items = list(data)
    back = IntervalData.from_items(items)
    for f in ('chrom', 'start', 'end', 'aln_size', 'n_alignments', 'qlen2', 'middle'):
        np.testing.assert_array_equal(getattr(back, f), getattr(data, f))
    assert [back.qnames[c] for c in back.qcode] == [data.qnames[c] for c in data.qcode]
    a, b = back.csr(), data.csr()
    for f in ('read_off', 'read_qlen2', 'read_nal', 'iv_chrom', 'iv_start', 'iv_end', 'iv_aln', 'data_pos'):
        np.testing.assert_array_equal(getattr(a, f), getattr(b, f))
    assert list(back.qnames[a.read_qcode]) == list(data.qnames[b.read_qcode])


def test_split_long_reads_layout():
    """The virtual CSR of the long-read stage: reads < n keep their first 64
    intervals, the further chunks follow in rank order, and every interval appears once."""
    from fslr_amd import synth
    from fslr_amd.prep import split_long_reads, has_long_reads
    csr = synth.generate(500, 200, 9, lmin=1).interval_data().csr()
    assert has_long_reads(csr)
    v, vreal, vbase, rlen = split_long_reads(csr)
    n = csr.n_reads
    np.testing.assert_array_equal(rlen, np.diff(csr.read_off))
    np.testing.assert_array_equal(vreal[:n], np.arange(n))
    vl = np.diff(v.read_off)
    assert vl.min() >= 1 and vl.max() <= 64
    assert np.all(np.diff(vreal[n:]) >= 0)
    # every virtual interval maps back to (real read, index) of the real CSR, each exactly once
    seen = np.zeros(csr.n_intervals, bool)
    for r in range(v.n_reads):
        for t in range(vl[r]):
            k = csr.read_off[vreal[r]] + vbase[r] + t
            assert not seen[k]
            seen[k] = True
            kv = v.read_off[r] + t
            assert (v.iv_start[kv], v.iv_end[kv], v.data_pos[kv]) == (csr.iv_start[k], csr.iv_end[k], csr.data_pos[k])
    assert seen.all()
    np.testing.assert_array_equal(v.read_qlen2, csr.read_qlen2[vreal])


def test_umax_table_matches_pass_table():
    from fslr_amd.prep import pass_table, umax_table
    for cut in ([1, 1, .66, .66, .66, .5], [0.3], [1.2], [0.0], [0.7, 0.2]):
        u = umax_table(cut, 64)
        pt = pass_table(cut).reshape(64, 128)
        for I in range(1, 65):
            ok = [U for U in range(I, 129) if pt[I - 1, U - 1]]
            assert u[I - 1] == min(max(ok) if ok else I - 1, 128)


@pytest.mark.parametrize('overlap', [0.8, 0.0, -0.5, 1.0, 0.33, 1.5])
def test_fold_lookup_table_path_equals_direct(overlap):
    """Large inputs fold each distinct value once (a lookup table gathered by value); the result equals
    the direct per-element fold, zeros included."""
    rng = np.random.default_rng(5)
    x = rng.integers(0, 6000, 300_000)
    x[::97] = 0
    big = fold_overlap_threshold(x, overlap)
    small = np.concatenate([fold_overlap_threshold(x[i:i + 50_000], overlap) for i in range(0, x.size, 50_000)])
    assert big.dtype == small.dtype
    np.testing.assert_array_equal(big, small)
