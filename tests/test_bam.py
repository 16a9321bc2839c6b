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


def _asan_driver(tmp_path):
    """tests/native/bam_asan_driver.cpp + bam.cpp built with -fsanitize=address (host code only)."""
    import shutil
    import subprocess
    if shutil.which('g++') is None:
        pytest.skip('no g++')
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = tmp_path / 'bam_asan'
    subprocess.run(['g++', '-O1', '-g', '-std=c++17', '-fsanitize=address,undefined', '-fno-omit-frame-pointer',
                    '-pthread', '-I' + os.path.join(root, 'include'), '-o', str(exe),
                    os.path.join(root, 'tests', 'native', 'bam_asan_driver.cpp'),
                    os.path.join(root, 'fslr_amd', 'csrc', 'bam.cpp'), '-lz'], check=True)
    return exe


def _corrupt_bams(tmp_path):
    """A valid BAM, then truncations of its BGZF file and of its decompressed stream, and records whose
    name / CIGAR / sequence / tag lengths point past their end."""
    import struct
    recs = [dict(qname=f'r{i}', flag=0, tid=i % 2, pos=10 * i, mapq=60, cigar=[('S', 3), ('M', 20), ('I', 2), ('M', 5)],
                 seq='ACGT' * 7 + 'A' * 3, tags=[('XA', 'Z', 'chr1,+5,10M,0'), ('AS', 'i', -i)]) for i in range(40)]
    good = tmp_path / 'good.bam'
    B.write_bam(str(good), [('chrA', 100000), ('chrB', 200000)], recs)
    raw = good.read_bytes()
    body = gzip.decompress(raw)
    files = [good]

    def put(name, data, compressed=False):
        p = tmp_path / name
        p.write_bytes(data if compressed else B._bgzf_block(bytes(data)) + B._BGZF_EOF)
        files.append(p)

    for cut in (5, 17, 18, 30, len(raw) // 2, len(raw) - 29, len(raw) - 1):
        put(f'ctrunc{cut}.bam', raw[:cut], compressed=True)
    blk = bytearray(raw)
    blk[10:12] = struct.pack('<H', 60000)            # XLEN past the file
    put('xlen.bam', blk, compressed=True)
    blk = bytearray(raw)
    blk[14:16] = struct.pack('<H', 400)              # the BC subfield's SLEN past XLEN
    put('slen.bam', blk, compressed=True)
    blk = bytearray(raw)
    blk[16:18] = struct.pack('<H', 3)                # BSIZE below header + trailer
    put('bsize.bam', blk, compressed=True)
    # the first record: its block_size field offset
    l_text = struct.unpack_from('<i', body, 4)[0]
    p = 8 + l_text
    n_ref = struct.unpack_from('<i', body, p)[0]
    p += 4
    for _ in range(n_ref):
        p += 8 + struct.unpack_from('<i', body, p)[0]
    r0 = p
    bs = struct.unpack_from('<i', body, r0)[0]
    for cut in (r0 + 20, r0 + 40, r0 + 4 + bs - 3, len(body) - 5):
        put(f'btrunc{cut}.bam', body[:cut])
    for name, off, fmt, val in [('lname0', 12, '<B', 0), ('ncig', 16, '<H', 4000), ('lseq', 20, '<i', 1 << 20),
                                ('lseqneg', 20, '<i', -7), ('bsneg', 0, '<i', -4), ('bsbig', 0, '<i', 1 << 30)]:
        b = bytearray(body)
        struct.pack_into(fmt, b, r0 + off, val)
        put(f'{name}.bam', b)
    # tags: the record's tag area starts after qual; corrupt the AS tag type and a B array count
    rec = body[r0:r0 + 4 + bs]
    t = rec.find(b'ASi')
    for name, patch in [('tagB', b'ASBi' + struct.pack('<i', -3)), ('tagBbig', b'ASBc' + struct.pack('<i', 1 << 28)),
                        ('tagtype', b'ASq'), ('tagZ', b'AS' + b'Z' + b'x' * 3)]:
        b = bytearray(body)
        seg = bytearray(rec)
        seg[t:t + len(patch)] = patch[:len(seg) - t]
        b[r0:r0 + 4 + bs] = seg[:4 + bs]
        put(f'{name}.bam', b)
    return files


def test_corrupt_bam_returns_an_error_under_asan(tmp_path):
    """Truncated or corrupt BAM / BGZF input: the decoder returns FSLR_BAM_ERROR instead of reading
    past its buffers (AddressSanitizer + UBSan build of bam.cpp)."""
    import subprocess
    exe = _asan_driver(tmp_path)
    files = _corrupt_bams(tmp_path)
    env = dict(os.environ, ASAN_OPTIONS='detect_leaks=0:abort_on_error=1', UBSAN_OPTIONS='halt_on_error=1')
    res = subprocess.run([str(exe)] + [str(f) for f in files], capture_output=True, text=True, env=env, timeout=120)
    assert res.returncode == 0, res.stderr[-3000:]
    lines = res.stdout.splitlines()
    assert len(lines) == len(files)
    assert lines[0] == 'ok 40'
    bad = dict(zip([f.name for f in files], lines))
    for name in ('xlen.bam', 'slen.bam', 'bsize.bam', 'lname0.bam', 'ncig.bam', 'lseq.bam', 'lseqneg.bam', 'bsneg.bam',
                 'bsbig.bam', 'tagB.bam', 'tagBbig.bam', 'tagtype.bam'):
        assert bad[name].startswith('error'), (name, bad[name])
