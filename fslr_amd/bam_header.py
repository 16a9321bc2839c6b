"""Minimal BGZF / BAM header reader and writer.

Replaces the one pysam call on the clustering path, ``cluster.get_chromosome_lengths``
(``cluster.py:173-175``: ``pysam.AlignmentFile(bam).lengths`` keyed by reference
name).  pysam is not installed in this image, and the path only needs the
header's reference dictionary, so the header is decoded directly:

    BGZF = concatenated gzip members (RFC 1952) carrying a ``BC`` extra subfield;
    BAM  = magic ``BAM\\1``, int32 l_text, text, int32 n_ref,
           n_ref × (int32 l_name, name\\0, int32 l_ref)     (SAMv1 §4.2).

Python's ``gzip`` reader accepts multi-member streams, so decoding is a plain
``gzip.open`` read of the leading bytes.  ``write_bam_header`` emits a valid
header-only BAM (header block + the 28-byte BGZF EOF marker) for fixtures.
"""
from __future__ import annotations

import gzip
import struct
import zlib

_BGZF_EOF = bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")


class BamHeaderError(ValueError):
    pass


def read_bam_references(path: str) -> list:
    """Return ``[(name, length), ...]`` in header (tid) order."""
    with gzip.open(path, 'rb') as fh:
        def take(n):
            b = fh.read(n)
            if len(b) != n:
                raise BamHeaderError(f"{path}: truncated BAM header")
            return b
        if take(4) != b"BAM\x01":
            raise BamHeaderError(f"{path}: not a BAM file (bad magic)")
        (l_text,) = struct.unpack('<i', take(4))
        take(l_text)
        (n_ref,) = struct.unpack('<i', take(4))
        refs = []
        for _ in range(n_ref):
            (l_name,) = struct.unpack('<i', take(4))
            name = take(l_name).rstrip(b'\x00').decode()
            (l_ref,) = struct.unpack('<i', take(4))
            refs.append((name, l_ref))
        return refs


def get_chromosome_lengths(bam_path: str) -> dict:
    """``{reference name: length}`` (cluster.py:173-175 semantics)."""
    return {name: length for name, length in read_bam_references(bam_path)}


def _bgzf_block(payload: bytes) -> bytes:
    comp = zlib.compressobj(6, zlib.DEFLATED, -15)
    data = comp.compress(payload) + comp.flush()
    bsize = 12 + 6 + len(data) + 8       # header(12) + extra(6) + cdata + crc/isize(8)
    head = struct.pack('<BBBBIBBH', 0x1f, 0x8b, 8, 4, 0, 0, 0xff, 6)
    extra = struct.pack('<BBHH', ord('B'), ord('C'), 2, bsize - 1)
    tail = struct.pack('<II', zlib.crc32(payload) & 0xffffffff, len(payload) & 0xffffffff)
    return head + extra + data + tail


def write_bam_header(path: str, references, text: str | None = None) -> None:
    """Write a header-only BAM with ``references`` = iterable of ``(name, length)``."""
    refs = list(references)
    if text is None:
        text = "@HD\tVN:1.6\tSO:coordinate\n" + "".join(f"@SQ\tSN:{n}\tLN:{l}\n" for n, l in refs)
    tb = text.encode()
    body = b"BAM\x01" + struct.pack('<i', len(tb)) + tb + struct.pack('<i', len(refs))
    for name, length in refs:
        nb = name.encode() + b'\x00'
        body += struct.pack('<i', len(nb)) + nb + struct.pack('<i', int(length))
    out = b""
    for i in range(0, len(body), 60000):
        out += _bgzf_block(body[i:i + 60000])
    with open(path, 'wb') as fh:
        fh.write(out + _BGZF_EOF)
