"""The `.mappings.bed` producer against the reference's own outputs.

tests/golden/bam/ holds a synthetic BAM and what the reference's collect_mapping_info.mapping_info
wrote for it (tests/golden/make_bam_golden.py, run through refharness' pysam stand-in).  Host
code only (libfslr_bam.so: zlib + C++), so these run on the CPU.
"""
import contextlib
import gzip
import io
import json
import os

import numpy as np
import pytest

from fslr_amd import bam as B
from fslr_amd import collect_mapping_info as CMI

GOLD = os.path.join(os.path.dirname(__file__), 'golden', 'bam')


def _meta():
    with open(os.path.join(GOLD, 'producer.json')) as fh:
        return json.load(fh)


@pytest.mark.parametrize('regions', [False, True])
@pytest.mark.parametrize('threads', [1, 4])
def test_mapping_info_matches_reference_output(tmp_path, regions, threads):
    out = tmp_path / 'x.mappings.bed'
    CMI.mapping_info(os.path.join(GOLD, 'input.bam'), str(out), os.path.join(GOLD, 'regions.bed') if regions else None,
                     _meta()['primers'], n_threads=threads)
    name = 'expected_regions.mappings.bed.gz' if regions else 'expected.mappings.bed.gz'
    assert out.read_bytes() == gzip.open(os.path.join(GOLD, name)).read()


def test_flag_problem_quits_like_the_reference(tmp_path):
    meta = _meta()
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf), pytest.raises(SystemExit) as e:
        CMI.mapping_info(os.path.join(GOLD, 'flag_problem.bam'), str(tmp_path / 'u.bed'), None, meta['primers'])
    assert e.value.code == meta['flag_problem_exit']
    assert buf.getvalue() == meta['flag_problem_stdout'].replace('{DIR}', GOLD)
    assert not (tmp_path / 'u.bed').exists()


def test_decoder_round_trips_written_records(tmp_path):
    """BamFile decodes what write_bam encodes: CIGAR-derived spans and clips, flags, AS, SEQ."""
    recs = [dict(qname='a.21q1F_17p6R', flag=0, tid=1, pos=99, mapq=60, cigar=[('S', 5), ('M', 10), ('D', 2), ('M', 3),
                                                                              ('I', 4), ('M', 6), ('H', 7)],
                 seq='ACGTACGTACGTACGTACGTACGTACGTA', tags=[('XA', 'Z', 'x'), ('AS', 'i', -3)]),
            dict(qname='b', flag=16 | 2048, tid=0, pos=0, mapq=1, cigar=[('H', 3), ('M', 4)], seq='AACG',
                 tags=[('AS', 'i', 70000)]),
            dict(qname='c', flag=4, tid=-1, pos=-1, mapq=0, cigar=[], seq='', tags=[])]
    p = tmp_path / 't.bam'
    B.write_bam(str(p), [('chrA', 1000), ('chrB', 2000)], recs)
    with B.BamFile(str(p), 2) as f:
        c = f.columns
        assert f.references == ['chrA', 'chrB'] and f.lengths == [1000, 2000]
        assert list(f.qname) == ['a.21q1F_17p6R', 'b', 'c']
        np.testing.assert_array_equal(c['flag'], [0, 2064, 4])
        np.testing.assert_array_equal(c['pos'], [99, 0, -1])
        np.testing.assert_array_equal(c['ref_span'], [21, 4, 0])
        np.testing.assert_array_equal(c['read_len'], [5 + 10 + 3 + 4 + 6 + 7, 7, 0])
        np.testing.assert_array_equal(c['clip_first'], [5, 3, 0])
        np.testing.assert_array_equal(c['clip_last'], [7, 0, 0])
        np.testing.assert_array_equal(c['as_tag'][:2], [-3, 70000])
        np.testing.assert_array_equal(c['as_kind'], [1, 1, 0])
        assert f.forward_sequence(0) == recs[0]['seq']
        assert f.forward_sequence(1) == 'CGTT'          # reverse complement of AACG


def test_cli_entry_writes_the_same_file(tmp_path):
    out = tmp_path / 'cli.bed'
    CMI.main(['--bam', os.path.join(GOLD, 'input.bam'), '--out', str(out), '--primers', '21q1,17p6'])
    assert out.read_bytes() == gzip.open(os.path.join(GOLD, 'expected.mappings.bed.gz')).read()


def test_library_exports_every_declared_symbol():
    import re
    hdr = open(os.path.join(os.path.dirname(os.path.dirname(__file__)), 'include', 'fslr_bam.h')).read()
    names = set(re.findall(r'\b(fslr_bam_\w+)\s*\(', hdr))
    L = B.load()
    assert names and all(hasattr(L, n) for n in names)
