"""BAM records for the ``.mappings.bed`` producer.

:class:`BamFile` decodes a whole BAM natively (``libfslr_bam.so``, C ABI ``include/fslr_bam.h``:
threaded BGZF inflate + one indexing pass) into the per-record columns that
``collect_mapping_info.mapping_info`` reads through pysam in the reference
(``fslr/collect_mapping_info.py:7-17,23-99``).  :func:`write_bam` writes BAM files (BGZF blocks of
SAMv1 §4.2 records) for fixtures and synthetic inputs.
"""
from __future__ import annotations

import ctypes
import os
import struct

import numpy as np

from .bam_header import _BGZF_EOF, _bgzf_block

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'libfslr_bam.so')
CIGAR_OPS = 'MIDNSHP=X'
_SEQ_CODE = {c: i for i, c in enumerate('=ACMGRSVTWYHKDBN')}
_lib = None


def load(path: str = LIB_PATH):
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise FileNotFoundError(f'{path} is not built: run `make -C fslr_amd/csrc`')
    L = ctypes.CDLL(path)
    vp, i64, i32, cp = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_char_p
    sig = {
        'fslr_bam_open': (i32, [cp, i32, ctypes.POINTER(vp), cp, ctypes.c_size_t]),
        'fslr_bam_close': (None, [vp]),
        'fslr_bam_n_records': (i64, [vp]),
        'fslr_bam_n_refs': (i32, [vp]),
        'fslr_bam_ref_name': (cp, [vp, i32]),
        'fslr_bam_ref_len': (i64, [vp, i32]),
        'fslr_bam_qname_bytes': (i64, [vp]),
        'fslr_bam_columns': (i32, [vp] + [vp] * 14),
        'fslr_bam_forward_seq': (i32, [vp, i64, vp]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype, f.argtypes = res, args
    _lib = L
    return L


class BamFile:
    """A decoded BAM: header references and per-record columns (file order)."""

    def __init__(self, path: str, n_threads: int = 0):
        L = load()
        err = ctypes.create_string_buffer(512)
        h = ctypes.c_void_p()
        if L.fslr_bam_open(os.fsencode(path), int(n_threads), ctypes.byref(h), err, len(err)) != 0:
            raise OSError(err.value.decode() or f'cannot decode {path}')
        self._h, self._L = h, L
        self.references = [L.fslr_bam_ref_name(h, t).decode() for t in range(L.fslr_bam_n_refs(h))]
        self.lengths = [int(L.fslr_bam_ref_len(h, t)) for t in range(len(self.references))]
        n = int(L.fslr_bam_n_records(h))
        self.n = n
        c = {k: np.empty(n, dtype=t) for k, t in (
            ('flag', np.int32), ('tid', np.int32), ('pos', np.int64), ('mapq', np.int32), ('ref_span', np.int64),
            ('read_len', np.int64), ('clip_first', np.int64), ('clip_last', np.int64), ('n_cigar', np.int32),
            ('as_tag', np.int64), ('as_kind', np.int8), ('l_seq', np.int64), ('qname_end', np.int64))}
        buf = ctypes.create_string_buffer(max(1, int(L.fslr_bam_qname_bytes(h))))
        order = ('flag', 'tid', 'pos', 'mapq', 'ref_span', 'read_len', 'clip_first', 'clip_last', 'n_cigar',
                 'as_tag', 'as_kind', 'l_seq', 'qname_end')
        if L.fslr_bam_columns(h, *[c[k].ctypes.data for k in order], buf) != 0:
            raise OSError(f'{path}: malformed alignment record')
        self.columns = c
        raw = buf.raw
        ends = c['qname_end']
        starts = np.concatenate(([0], ends[:-1])) if n else ends
        self.qname = np.array([raw[s:e].decode() for s, e in zip(starts.tolist(), ends.tolist())], dtype=object)

    def forward_sequence(self, rec: int) -> str:
        """pysam ``get_forward_sequence()`` of record ``rec`` ('' for SEQ '*')."""
        n = int(self.columns['l_seq'][rec])
        out = ctypes.create_string_buffer(max(1, n))
        if self._L.fslr_bam_forward_seq(self._h, int(rec), out) != 0:
            raise IndexError(rec)
        return out.raw[:n].decode()

    def close(self):
        if self._h is not None:
            self._L.fslr_bam_close(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ------------------------------------------------------------------ writing (fixtures)
def encode_record(qname: str, flag: int, tid: int, pos: int, mapq: int, cigar, seq: str, tags=()) -> bytes:
    """One SAMv1 §4.2 alignment record.  ``cigar``: [(op letter, length)]; ``tags``: [(name, type, value)]
    with type 'i' (int32) or 'Z' (string)."""
    name = qname.encode() + b'\0'
    cg = b''.join(struct.pack('<I', (n << 4) | CIGAR_OPS.index(op)) for op, n in cigar)
    ls = len(seq)
    packed = bytearray((ls + 1) // 2)
    for i, ch in enumerate(seq):
        packed[i >> 1] |= _SEQ_CODE[ch] << (4 if i % 2 == 0 else 0)
    qual = b'\xff' * ls
    tb = b''
    for tname, ttype, val in tags:
        if ttype == 'i':
            tb += tname.encode() + b'i' + struct.pack('<i', int(val))
        elif ttype == 'Z':
            tb += tname.encode() + b'Z' + str(val).encode() + b'\0'
        elif ttype == 'f':
            tb += tname.encode() + b'f' + struct.pack('<f', float(val))
        else:
            raise ValueError(ttype)
    body = struct.pack('<iiBBHHHiiii', tid, pos, len(name), mapq, 4680, len(cigar), flag, ls, -1, -1, 0)
    body += name + cg + bytes(packed) + qual + tb
    return struct.pack('<i', len(body)) + body


def write_bam(path: str, references, records) -> None:
    """Write a BAM: ``references`` = [(name, length)], ``records`` = iterable of encode_record kwargs dicts."""
    refs = list(references)
    text = '@HD\tVN:1.6\n' + ''.join(f'@SQ\tSN:{n}\tLN:{l}\n' for n, l in refs)
    tb = text.encode()
    body = bytearray(b'BAM\x01' + struct.pack('<i', len(tb)) + tb + struct.pack('<i', len(refs)))
    for name, length in refs:
        nb = name.encode() + b'\0'
        body += struct.pack('<i', len(nb)) + nb + struct.pack('<i', int(length))
    for r in records:
        body += encode_record(**r)
    with open(path, 'wb') as fh:
        for i in range(0, len(body), 60000):
            fh.write(_bgzf_block(bytes(body[i:i + 60000])))
        fh.write(_BGZF_EOF)
