"""The clustering input made on the device from rows (fslr_set_reads_rows): the
`data` list (prepare_data's start order, mask_sequences2 as keep flags; cluster.py:89-121), the read
ranks by first appearance and each read's intervals in data order (cluster.py:189-191), the dense
chromosome ids and the folded overlap thresholds (cluster.py:133-136) must equal what the host builds
(prep.build_csr, prep.fold_overlap_threshold) from the same rows — bit for bit — and the CLI outputs
stay the reference's.
"""
import os
import shutil
import tempfile

import numpy as np
import pytest

import fixtures as fx
from fslr_amd import _lib, cluster, synth
from fslr_amd.prep import fold_overlap_threshold

pytestmark = pytest.mark.gpu

CSR_FIELDS = ('read_off', 'read_qlen2', 'read_nal', 'iv_chrom', 'iv_start', 'iv_end', 'iv_aln', 'data_pos',
              'read_qcode')


def _check_rows_index(monkeypatch, seen):
    """Wrap RowsIndex so every device-built input is compared with the host build of the same rows."""
    orig = cluster.RowsIndex.__init__

    def wrapped(self, data, csr, ctx, overlap):
        h = data.csr()                                   # the host path: gathers + prep.build_csr
        d = csr.host()
        for k in CSR_FIELDS:
            np.testing.assert_array_equal(np.asarray(getattr(d, k), np.int64), np.asarray(getattr(h, k), np.int64),
                                          err_msg=k)
        assert d.n_chroms == h.n_chroms and d.nal_varies == h.nal_varies
        thr = ctx.device_csr(csr.n_intervals, csr.n_chroms)['iv_thr']
        np.testing.assert_array_equal(thr, fold_overlap_threshold(h.iv_aln, overlap))
        seen.append(csr.n_reads)
        orig(self, data, csr, ctx, overlap)
    monkeypatch.setattr(cluster.RowsIndex, '__init__', wrapped)


def _cli(bed_text, bam, args, tmp):
    from click.testing import CliRunner
    from fslr_amd.main import pipeline
    with open(os.path.join(tmp, 'fx.mappings.bed'), 'w') as fh:
        fh.write(bed_text)
    shutil.copy(bam, os.path.join(tmp, 'fx.bwa_dodi.bam'))
    argv = ['--name', 'fx', '--out', tmp, '--ref', 'unused.fa', '--primers', '21q1', '--skip-alignment',
            '--timings'] + list(args) + ['--native-io']
    return CliRunner().invoke(pipeline, argv, catch_exceptions=True)


@pytest.mark.parametrize('name', list(fx.FIXTURES))
def test_rows_input_equals_host_build_and_outputs_match(name, monkeypatch):
    seen = []
    _check_rows_index(monkeypatch, seen)
    meta = fx.meta(name)
    with tempfile.TemporaryDirectory() as tmp:
        res = _cli(fx.input_bed_text(name), fx.input_bam(name), meta['args'], tmp)
        if meta['exception']:
            assert isinstance(res.exception, ZeroDivisionError), res.output
            return
        assert res.exit_code == 0, (res.output, res.exception)
        for which in ('cluster', 'representative'):
            want = fx.expected_text(name, which)
            path = os.path.join(tmp, f'fx.mappings.{which}.bed')
            assert (open(path).read() if os.path.exists(path) else None) == want, which
    long_reads = name.startswith('long') or name in ('longreads_400',) or name.endswith('_long')
    if 'path=columns' in res.output and not long_reads:
        assert seen, 'the columnar path did not build its input on the device'


def test_rows_ties_and_mask_200k(monkeypatch):
    """Many equal starts (pandas' quicksort tie order decides the read ranks) and subtelomere masking on
    a 200k-read input: the device's ranks and lists equal the host's."""
    seen = []
    _check_rows_index(monkeypatch, seen)
    s = synth.generate(200_000, 16, 5)
    df = s.to_dataframe()
    fill = df['aln_size'] != 20
    st = df.loc[fill, 'rstart'].to_numpy()
    df.loc[fill, 'rstart'] = (st // 5000) * 5000                   # coarse grid: most starts tie
    df.loc[fill, 'rend'] = df.loc[fill, 'rstart'] + df.loc[fill, 'aln_size']
    from fslr_amd import bam_header
    with tempfile.TemporaryDirectory() as tmp:
        bam = os.path.join(tmp, 'h.bam')
        bam_header.write_bam_header(bam, s.chrom_lengths.items())
        res = _cli(df.to_csv(sep='\t', index=False), bam, [], tmp)
        assert res.exit_code == 0, (res.output, res.exception)
    assert seen == [seen[0]] and seen[0] > 100_000


@pytest.mark.parametrize('overlap', [0.8, 0.5, 0.95, 1.0, 1e-9, 0.3333333333333333, 0.0, -0.5, -1.0, 2.0])
def test_device_threshold_fold_equals_host(overlap):
    """fold_overlap_threshold on the device (rows.hip fold_one) for aln_size values at the edges of the
    integer fold: 0 (ZeroDivisionError marker), 1, 2, 3, primes, powers of two, 2^29 .. 2^31 - 1, and
    negative values; then fslr_fold_thresholds for every other overlap."""
    alns = np.array([0, 1, 2, 3, 5, 7, 97, 100, 101, 1000, 4093, 65536, 12345, 999_983, 1 << 20, (1 << 29) - 1,
                     1 << 29, (1 << 30) - 3, (1 << 31) - 1, -1, -7, -100, -(1 << 29)], np.int64)
    n = alns.size
    rows = dict(chrom=np.ones(n, np.int64), start=np.arange(n, dtype=np.int64) * 10,
                end=np.arange(n, dtype=np.int64) * 10 + 5, aln=alns, qcode=np.arange(n, dtype=np.int64),
                nal=np.full(n, 3, np.int64), qlen2=np.full(n, 100, np.int64))
    ctx = _lib.Context(0)
    try:
        ctx.rows_upload(rows, n, 2)
        info = ctx.set_reads_rows(np.arange(n, dtype=np.int64), None, overlap)
        assert info['n_reads'] == n and info['n_intervals'] == n
        d = ctx.device_csr(n, info['n_chroms'])
        np.testing.assert_array_equal(d['iv_aln'], alns)
        np.testing.assert_array_equal(d['iv_thr'], fold_overlap_threshold(alns, overlap))
        for p in (0.8, 0.0, -0.25, 0.5000000001):
            ctx.fold_thresholds(p)
            np.testing.assert_array_equal(ctx.device_csr(n, info['n_chroms'])['iv_thr'],
                                          fold_overlap_threshold(alns, p))
    finally:
        ctx.close()


def test_rows_long_read_declined():
    """A read of more than FSLR_MAX_L intervals: nothing is set, the info names the length (the CLI then
    builds the CSR on the host and uploads it with fslr_set_reads_any)."""
    n = 70
    rows = dict(chrom=np.ones(n, np.int64), start=np.arange(n, dtype=np.int64) * 10,
                end=np.arange(n, dtype=np.int64) * 10 + 5, aln=np.full(n, 5, np.int64),
                qcode=np.zeros(n, np.int64), nal=np.full(n, 3, np.int64), qlen2=np.full(n, 100, np.int64))
    ctx = _lib.Context(0)
    try:
        ctx.rows_upload(rows, 1, 2)
        with pytest.raises(_lib.FslrError) as e:
            ctx.set_reads_rows(np.arange(n, dtype=np.int64), None, 0.8)
        assert e.value.info['max_len'] == n
    finally:
        ctx.close()


def _jittered_rows(n_reads, seed):
    """Rows of reads with 1-4 intervals of ~1 kb whose starts are jittered by up to 700 bp around shared
    loci, so the reciprocal overlaps spread over 0.3-1.0 (overlap 0.5 and 0.8 give different graphs)."""
    rng = np.random.default_rng(seed)
    L = rng.integers(1, 5, n_reads)
    q = np.repeat(np.arange(n_reads, dtype=np.int64), L)
    m = q.size
    locus = rng.integers(0, 400, m) * 5000
    start = locus + rng.integers(0, 700, m)
    size = rng.integers(900, 1100, m)
    rows = dict(chrom=rng.integers(1, 3, m).astype(np.int64), start=start.astype(np.int64),
                end=(start + size).astype(np.int64), aln=size.astype(np.int64), qcode=q,
                nal=np.repeat(L, L).astype(np.int64), qlen2=np.full(m, 5000, np.int64))
    return rows, n_reads


def _edge_set(ctx, st):
    a, b, I, U = ctx.edges(st['n_edges'])
    return sorted(zip(a.tolist(), b.tolist(), I.tolist(), U.tolist()))


@pytest.mark.parametrize('engine', ['sweep', 'walk'])
def test_rows_index_refolded_overlap_queries_new_windows(engine):
    """A RowsIndex built (and its sweep windows cut) at overlap 0.8, then queried at 0.5 through
    fslr_fold_thresholds: the windows follow the new thresholds (start_p <= end_q - thr_q), so the
    edges equal a host-CSR context queried at 0.5 from the start (the fold left the
    windows at 0.8's and the sweep dropped pairs silently)."""
    from fslr_amd.prep import pass_table
    rows, n = _jittered_rows(3000, 21)
    order = np.argsort(rows['start'], kind='stable').astype(np.int64)
    pt = pass_table([0.3] * 8)
    r = _lib.Context(0)
    h = _lib.Context(0)
    try:
        r.rows_upload(rows, n, 3)
        info = r.set_reads_rows(order, None, 0.8)
        r.reserve_edges(1 << 18)
        r.build_index()
        st8 = r.run_query(0.0, 0.0, pt, engine=engine)
        e8 = _edge_set(r, st8)
        r.fold_thresholds(0.5)
        st5 = r.run_query(0.0, 0.0, pt, engine=engine)
        e5 = _edge_set(r, st5)
        d = r.device_csr(info['n_intervals'], info['n_chroms'])
        h.set_reads(d['read_off'], d['read_qlen2'], d['read_nal'], d['iv_chrom'], d['iv_start'], d['iv_end'],
                    fold_overlap_threshold(d['iv_aln'], 0.5), info['n_chroms'], iv_data_pos=d['data_pos'])
        h.reserve_edges(1 << 18)
        h.build_index()
        sth = h.run_query(0.0, 0.0, pt, engine=engine)
        assert len(e5) > len(e8) > 0
        assert e5 == _edge_set(h, sth)
    finally:
        r.close()
        h.close()


def test_rows_code_out_of_range_is_invalid_not_a_fault():
    """A qname code outside [0, n_codes) is reported as FSLR_ERR_INVALID before the grouping reads the
    ranks (k_rows_isfirst / k_rows_rank read first[q] out of bounds); the context then takes
    a valid upload."""
    rows, n = _jittered_rows(200, 3)
    order = np.argsort(rows['start'], kind='stable').astype(np.int64)
    ctx = _lib.Context(0)
    try:
        for bad in (n, n + 1000, -5):
            r2 = dict(rows, qcode=rows['qcode'].copy())
            r2['qcode'][7] = bad
            ctx.rows_upload(r2, n, 3)
            with pytest.raises(_lib.FslrError, match='qname code out of range'):
                ctx.set_reads_rows(order, None, 0.8)
        ctx.rows_upload(rows, n, 3)
        assert ctx.set_reads_rows(order, None, 0.8)['n_reads'] == n
    finally:
        ctx.close()
