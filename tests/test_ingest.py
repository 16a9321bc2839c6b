"""Native `.mappings.bed` reader (fslr_amd/ingest.py, include/fslr_ingest.h) against pandas.

The oracle here is pandas itself: ``pd.read_csv(path, sep='\\t', usecols=HOT_COLUMNS)`` is what the
reference does at fslr/main.py:209.  Every golden input must come back identical (values, dtypes,
column order); inputs pandas would type differently must be declined (None), never mis-typed.
"""
import gzip
import glob
import os

import pandas as pd
import numpy as np
import pytest

from fslr_amd import ingest

GOLDEN = os.path.join(os.path.dirname(__file__), 'golden')
HEADER = 'chrom\trstart\trend\tqname\tn_alignments\taln_size\tqstart\tqend\tstrand\tseq\n'


def _ref(path):
    return pd.read_csv(path, sep='\t', usecols=list(ingest.HOT_COLUMNS))


@pytest.mark.parametrize('src', sorted(glob.glob(os.path.join(GOLDEN, '*', 'input.mappings.bed.gz'))),
                         ids=lambda p: os.path.basename(os.path.dirname(p)))
@pytest.mark.parametrize('threads', [1, 3, 8])
def test_golden_inputs_match_pandas(tmp_path, src, threads):
    p = tmp_path / 'x.mappings.bed'
    p.write_bytes(gzip.open(src).read())
    got = ingest.read_hot_columns(str(p), threads)
    ref = _ref(p)
    assert got is not None
    assert list(got.columns) == list(ref.columns)
    assert dict(got.dtypes) == dict(ref.dtypes)
    assert got.equals(ref)


def _rows(n, qname=lambda i: f'r{i // 3}', chrom=lambda i: f'chr{1 + i % 4}'):
    return ''.join(f'{chrom(i)}\t{100 * i}\t{100 * i + 50}\t{qname(i)}\t5\t50\t{10 * i}\t{10 * i + 50}\t+\tAC\n'
                   for i in range(n))


@pytest.mark.parametrize('body', [
    _rows(50),
    _rows(50).replace('\n', '\r\n'),                       # CRLF
    _rows(50)[:-1],                                        # no trailing newline
    _rows(20) + '\n\n' + _rows(20) + '\n',                 # blank lines are skipped
    _rows(9000, qname=lambda i: f'read{(i * 7919) % 1000}'),  # chunked factorize, non-adjacent repeats
    '',                                                    # header only
], ids=['plain', 'crlf', 'no_final_newline', 'blank_lines', 'scattered_qnames', 'empty'])
@pytest.mark.parametrize('threads', [1, 4])
def test_layout_edge_cases_match_pandas(tmp_path, body, threads):
    p = tmp_path / 'x.bed'
    p.write_text(HEADER + body, newline='')
    got = ingest.read_hot_columns(str(p), threads)
    ref = _ref(p)
    if len(ref) == 0:
        # pandas gives object dtype for every column of an empty frame; the fast path declines it
        # (all-int test is vacuous) or returns the same empty columns.
        assert got is None or len(got) == 0
        return
    assert got is not None and got.equals(ref) and dict(got.dtypes) == dict(ref.dtypes)


@pytest.mark.parametrize('mutate', [
    lambda s: s.replace('\t5\t50\t', '\t5\t050\t', 1),     # leading zero: pandas int 50, would write "50"
    lambda s: s.replace('\t5\t50\t', '\t5\t50.0\t', 1),    # float column
    lambda s: s.replace('\t5\t50\t', '\t5\t\t', 1),        # missing value -> float64 NaN
    lambda s: s.replace('r0\t', 'NA\t', 1),                # NA spelling in a string column
    lambda s: s.replace('r0\t', '"r0"\t', 1),              # quoting
    lambda s: s.replace('chr1\t', '1\t').replace('chr2\t', '2\t').replace('chr3\t', '3\t').replace('chr4\t', '4\t'),
], ids=['leading_zero', 'float', 'missing', 'na_string', 'quoted', 'all_int_chrom'])
def test_inputs_pandas_types_differently_are_declined(tmp_path, mutate):
    p = tmp_path / 'x.bed'
    p.write_text(mutate(HEADER + _rows(30)), newline='')
    assert ingest.read_hot_columns(str(p), 2) is None


@pytest.mark.parametrize('text', [
    HEADER + _rows(30).replace('\tAC\n', '\tAC\textra\n', 1),                       # a row wider than the header
    HEADER + _rows(30).replace('\t+\tAC\n', '\t+\n', 2),                             # rows narrower than it
    HEADER.replace('strand', 'seq') + _rows(30),                                    # repeated name -> 'seq.1'
    HEADER.replace('strand', '') + _rows(30),                                       # empty name -> 'Unnamed: 8'
    HEADER + _rows(30).replace('\tAC\n', '\tACx\n').replace('\tACx\n', '\t12\n', 3),   # ints, then text
    HEADER + _rows(30).replace('\tAC\n', '\t7\n', 29),                               # text after 29 ints
    HEADER + _rows(30).replace('\tAC\n', '\t1.5\n', 1),                              # a float among text
], ids=['wide_row', 'short_rows', 'dup_name', 'empty_name', 'int_then_text', 'text_last', 'float_in_text'])
def test_verbatim_declines_rows_pandas_would_rewrite(tmp_path, text):
    """The writer copies input row bytes only when to_csv would write them unchanged: ragged rows
    and header names pandas renames send the CLI to the pandas path."""
    p = tmp_path / 'x.bed'
    p.write_text(text, newline='')
    t = ingest.TsvFile(str(p))
    try:
        assert t.declined or not t.verbatim()
    finally:
        t.close()


def test_verbatim_accepts_a_clean_file(tmp_path):
    p = tmp_path / 'x.bed'
    p.write_text(HEADER + _rows(30), newline='')
    t = ingest.TsvFile(str(p))
    try:
        assert not t.declined and t.verbatim()
    finally:
        t.close()


def test_library_exports_every_declared_symbol():
    L = ingest.load()
    hdr = open(os.path.join(os.path.dirname(__file__), '..', 'include', 'fslr_ingest.h')).read()
    import re
    names = set(re.findall(r'\b(fslr_tsv_\w+)\s*\(', hdr))
    assert names and all(hasattr(L, n) for n in names)


@pytest.mark.parametrize('name', ['cfg1_1k_x3', 'mixed_1500_l16', 'ties_600', 'edge_cases', 'zipf_800_l64'])
def test_clustering_input_from_native_columns_matches_pandas(tmp_path, name):
    """keep_fillings → prepare_data (cluster.py:14,109) read only HOT_COLUMNS, so the device input
    built from the native reader equals the one built from the full pandas frame."""
    import dataclasses
    import numpy as np
    import fixtures as fx
    from host_pipeline import host_prepare
    p = tmp_path / 'x.mappings.bed'
    p.write_text(fx.input_bed_text(name), newline='')
    native = ingest.read_hot_columns(str(p), 4)
    assert native is not None
    a, _, _ = host_prepare(name)
    b, _, _ = host_prepare(name, bed=native)
    for f in dataclasses.fields(a):
        if f.name == '_csr':
            continue
        x, y = getattr(a, f.name), getattr(b, f.name)
        assert x.dtype == y.dtype and np.array_equal(x, y), f.name
    ca, cb = a.csr(), b.csr()
    for f in dataclasses.fields(ca):
        assert np.array_equal(np.asarray(getattr(ca, f.name)), np.asarray(getattr(cb, f.name))), f.name


def _golden_with_outputs():
    out = []
    for d in sorted(glob.glob(os.path.join(GOLDEN, '*'))):
        if os.path.exists(os.path.join(d, 'expected.cluster.bed.gz')) and \
                os.path.exists(os.path.join(d, 'input.mappings.bed.gz')):
            out.append(os.path.basename(d))
    return out


@pytest.mark.parametrize('name', _golden_with_outputs())
@pytest.mark.parametrize('kind', ['cluster', 'representative'])
def test_writer_reproduces_reference_outputs_byte_exact(tmp_path, name, kind):
    """The reference's own `.mappings.{cluster,representative}.bed` (main.py to_csv) rebuilt from the
    input bytes + pandas-formatted per-qname suffix columns, byte for byte."""
    import io
    src = gzip.open(os.path.join(GOLDEN, name, 'input.mappings.bed.gz')).read()
    exp = gzip.open(os.path.join(GOLDEN, name, f'expected.{kind}.bed.gz')).read()
    p = tmp_path / 'in.bed'
    p.write_bytes(src)
    in_lines = src.decode().split('\n')[1:]
    pos = {ln: i for i, ln in enumerate(in_lines) if ln}
    n_in = len(in_lines[0].split('\t'))
    exp_df = pd.read_csv(io.BytesIO(exp), sep='\t', float_precision='round_trip')
    if len(exp_df) == 0:
        pytest.skip('empty output')
    rows = [pos['\t'.join(ln.split('\t')[:n_in])] for ln in exp.decode().split('\n')[1:] if ln]
    with ingest.TsvFile(str(p), 4) as t:
        if not t.verbatim():
            pytest.skip('input not verbatim-writable (pandas path)')
        o = tmp_path / 'out.bed'
        t.write_rows(str(o), rows, exp_df.iloc[:, n_in:], exp_df['qname'])
    assert o.read_bytes() == exp


@pytest.mark.parametrize('name', _golden_with_outputs())
def test_shared_qname_codes_match_pandas(tmp_path, name):
    """The reader's qname codes (ingest.QnameCodes in attrs) give pd.factorize(sort=False) of every
    frame the clustering block derives (keep_fillings' rows, the representative rows), and
    choose_alignment's bincount path equals pandas' groupby mean / idxmax on the reference's own
    cluster assignment (cluster.py:237-254)."""
    import io
    import numpy as np
    from fslr_amd import cluster
    src = gzip.open(os.path.join(GOLDEN, name, 'input.mappings.bed.gz')).read()
    exp = pd.read_csv(io.BytesIO(gzip.open(os.path.join(GOLDEN, name, 'expected.cluster.bed.gz')).read()), sep='\t')
    p = tmp_path / 'in.bed'
    p.write_bytes(src)
    with ingest.TsvFile(str(p), 3) as t:
        bed = ingest.frame_from(t, int_columns=ingest.INT_COLUMNS + ('alignment_score',))
    if bed is None or len(exp) == 0:
        pytest.skip('input declined by the native reader')
    assert isinstance(bed.attrs.get(ingest.ATTR), ingest.QnameCodes)
    rng = np.random.default_rng(5)
    subsets = [bed, bed[rng.random(len(bed)) < 0.5], cluster.keep_fillings(bed.copy())]
    for df in subsets:
        c1, u1 = ingest.factorize_qname(df)
        c2, u2 = pd.factorize(df['qname'], sort=False)
        assert np.array_equal(c1, c2) and list(u1) == list(u2)
    per_q = exp.drop_duplicates('qname').set_index('qname')
    for col in ('cluster', 'n_reads'):
        bed[col] = bed['qname'].map(per_q[col]).to_numpy()
    assert cluster._choose_alignment_codes(bed.copy()) is not None      # the bincount path runs
    plain = bed.copy()
    plain.attrs = {}
    fast = cluster.choose_alignment(bed)
    slow = cluster.choose_alignment(plain)
    assert fast.index.equals(slow.index)
    np.testing.assert_array_equal(fast['avg_alignment_score'].to_numpy(), slow['avg_alignment_score'].to_numpy())
    np.testing.assert_array_equal(bed['avg_alignment_score'].to_numpy(), plain['avg_alignment_score'].to_numpy())


def test_native_suffix_text_equals_pandas_to_csv():
    """fslr_format_suffix writes int64 and float64 columns exactly as DataFrame.to_csv does (numpy's
    str(): shortest round-trip digits, positional for exponents -4..15, '.0' when integral)."""
    import numpy as np
    rng = np.random.default_rng(1)
    vals = np.concatenate([rng.random(20000) * 10.0 ** rng.integers(-8, 20, 20000),
                           np.arange(-5, 3000, dtype=float),
                           rng.integers(0, 10 ** 6, 5000) / rng.integers(1, 1000, 5000),
                           [0.0, -0.0, 1e16, 1e15, 9999999999999998.0, 1e-4, 1e-5, 0.1, 0.3, 1 / 3, 2.0 ** 53,
                            1.5e300, 5e-324, 123456789.125, -2.5e-7, 45.0, 1234.5]])
    df = pd.DataFrame({'a': rng.integers(-10 ** 15, 10 ** 15, len(vals)), 'b': vals, 'c': vals * 3})
    buf, ends = ingest.format_suffix(df)
    text = df.to_csv(sep='\t', header=False, index=False, lineterminator='\n')
    assert buf == b''.join(('\t' + ln).encode() for ln in text.split('\n')[:len(df)])
    assert ends[-1] == len(buf)
    assert ingest.format_suffix(pd.DataFrame({'x': [1.0, float('nan')]})) is None        # na_rep: pandas
    assert ingest.format_suffix(pd.DataFrame({'x': ['a', 'b']})) is None


def test_argsort_distinct_radix_matches_numpy():
    """prepare_data's start order (cluster.py:114): the native radix argsort stands in for numpy's
    quicksort only when no two starts tie (then every sort agrees); a tie or a key range wider than
    2^32 hands the sort back to numpy, whose tie order is pandas'."""
    from fslr_amd import ingest
    from fslr_amd.prep import data_order
    rng = np.random.default_rng(5)
    for n in (1, 2, 1000, 70_000, 400_000):
        k = (rng.permutation(3 * n)[:n].astype(np.int64) - n) * 5
        o = ingest.argsort_distinct(k, n_threads=3)
        assert o is not None
        np.testing.assert_array_equal(o, np.argsort(k, kind='stable'))
        np.testing.assert_array_equal(data_order(k), np.argsort(k, kind='quicksort'))
    tied = rng.integers(0, 5000, 100_000)
    assert ingest.argsort_distinct(tied) is None
    np.testing.assert_array_equal(data_order(tied), tied.astype(np.int64).argsort(kind='quicksort'))
    assert ingest.argsort_distinct(np.array([0, 1 << 33], dtype=np.int64)) is None
