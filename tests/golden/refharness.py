"""Import the *reference* fslr (read-only at /root/reference) for golden-vector capture.

Test infrastructure only: used by ``make_golden.py`` and by the optional live
cross-check in ``tests/test_oracle_live.py``.  It never travels to the GPU box
(``/root/reference`` does not exist there) and nothing in the product imports it.

The reference imports packages that are not installed in this image
(SURVEY.md §8c): ``pysam``, ``superintervals`` (>= 0.2.10, unpinned, C++/Cython),
``skbio``.  They are replaced by stand-ins that restate only what the clustering
path needs:

* ``pysam.AlignmentFile(bam).lengths / .get_reference_name(tid)`` — the BAM
  header dictionary (``cluster.py:173-175``), decoded by ``fslr_amd.bam_header``;
  ``.fetch(until_eof=True)`` — records as ``_AlignedSegment`` stand-ins decoded in pure
  Python here (for ``collect_mapping_info.py``; independent of the product's C++ decoder).
* ``superintervals.IntervalMap`` — ``add(start, end, value)``, ``build()``,
  ``search_values(start, end)``: every stored interval with ``start <= qend and
  end >= qstart`` (end-inclusive).  Result ORDER is the library's undocumented
  behaviour; this stand-in returns hits in descending position of the
  ``(start asc, end desc, insertion)`` order.  Order only matters when the
  edge cap binds, so fixtures that depend on it are
  labelled "stub-order".
* ``skbio.alignment.StripedSmithWaterman`` — unused on the clustering path.
* ``importlib.metadata.version('fslr')`` → ``'0.3.10'`` (``setup.py:6``).
"""
from __future__ import annotations

import bisect
import importlib
import importlib.metadata
import os
import sys
import types

REF_ROOT = '/root/reference'
_loaded = {}


def available() -> bool:
    return os.path.isdir(os.path.join(REF_ROOT, 'fslr'))


class _IntervalMap:
    def __init__(self, *args, **kwargs):
        self._items = []
        self._built = False

    def add(self, start, end, value=None):
        self._items.append((start, end, len(self._items), value))
        self._built = False

    def build(self):
        self._items.sort(key=lambda t: (t[0], -t[1], t[2]))
        self._starts = [t[0] for t in self._items]
        self._pmax = []
        m = None
        for t in self._items:
            m = t[1] if m is None else max(m, t[1])
            self._pmax.append(m)
        self._built = True

    def search_values(self, start, end):
        if not self._built:
            self.build()
        hi = bisect.bisect_right(self._starts, end)
        out = []
        i = hi - 1
        while i >= 0 and self._pmax[i] >= start:
            s, e, _, v = self._items[i]
            if e >= start:
                out.append(v)
            i -= 1
        return out


class _AlignedSegment:
    """pysam.AlignedSegment stand-in for collect_mapping_info.py: the attributes it reads, decoded
    here in pure Python (struct) from SAMv1 §4.2, following pysam's documented semantics:
    infer_read_length = M I S = X H lengths, infer_query_length = M I S = X lengths,
    reference_end = reference_start + M D N = X lengths, get_forward_sequence = SEQ
    reverse-complemented (A<->T, C<->G) when flag & 16."""

    def __init__(self, **kw):
        self.__dict__.update(kw)

    @property
    def rname(self):
        return self.reference_id

    def infer_read_length(self):
        return sum(n for op, n in self.cigartuples if op in (0, 1, 4, 7, 8, 5))

    def infer_query_length(self):
        return sum(n for op, n in self.cigartuples if op in (0, 1, 4, 7, 8))

    @property
    def reference_end(self):
        return self.reference_start + sum(n for op, n in self.cigartuples if op in (0, 2, 3, 7, 8))

    def get_tag(self, name):
        if name not in self.tags:
            raise KeyError(f"tag '{name}' not present")
        return self.tags[name]

    def get_forward_sequence(self):
        s = self.seq
        if s is None:
            return None
        if self.flag & 16:
            s = s[::-1].translate(str.maketrans('ACGT', 'TGCA'))
        return s


def _read_records(path):
    import gzip
    import struct
    data = gzip.open(path, 'rb').read()
    (l_text,) = struct.unpack_from('<i', data, 4)
    p = 8 + l_text
    (n_ref,) = struct.unpack_from('<i', data, p)
    p += 4
    for _ in range(n_ref):
        (l_name,) = struct.unpack_from('<i', data, p)
        p += 8 + l_name
    out = []
    code = '=ACMGRSVTWYHKDBN'
    while p < len(data):
        (bs,) = struct.unpack_from('<i', data, p)
        (tid, pos, l_rn, mapq, _bin, n_cig, flag, l_seq, _nt, _np, _tl) = struct.unpack_from('<iiBBHHHiiii', data, p + 4)
        q = p + 36
        name = data[q:q + l_rn - 1].decode()
        q += l_rn
        cig = []
        for c in range(n_cig):
            (v,) = struct.unpack_from('<I', data, q + 4 * c)
            cig.append((v & 15, v >> 4))
        q += 4 * n_cig
        sb = data[q:q + (l_seq + 1) // 2]
        seq = ''.join(code[(sb[i // 2] >> (4 if i % 2 == 0 else 0)) & 15] for i in range(l_seq)) if l_seq else None
        q += (l_seq + 1) // 2 + l_seq
        end = p + 4 + bs
        tags = {}
        while q < end:
            tn = data[q:q + 2].decode()
            ty = chr(data[q + 2])
            q += 3
            if ty in 'cCsSiI':
                fmt = {'c': '<b', 'C': '<B', 's': '<h', 'S': '<H', 'i': '<i', 'I': '<I'}[ty]
                (v,) = struct.unpack_from(fmt, data, q)
                q += struct.calcsize(fmt)
            elif ty == 'f':
                (v,) = struct.unpack_from('<f', data, q)
                q += 4
            elif ty == 'A':
                v = chr(data[q])
                q += 1
            elif ty in 'ZH':
                z = data.index(b'\0', q)
                v = data[q:z].decode()
                q = z + 1
            else:
                raise ValueError(f'tag type {ty}')
            tags[tn] = v
        out.append(_AlignedSegment(qname=name, flag=flag, reference_id=tid, reference_start=pos, mapq=mapq,
                                   cigartuples=cig, seq=seq, tags=tags))
        p = end
    return out


def _install_stubs():
    from fslr_amd import bam_header

    pysam = types.ModuleType('pysam')

    class AlignmentFile:
        def __init__(self, path, mode='rb', *a, **k):
            refs = bam_header.read_bam_references(path)
            self._path = path
            self._names = [n for n, _ in refs]
            self.lengths = tuple(l for _, l in refs)
            self.references = tuple(self._names)

        def get_reference_name(self, tid):
            return self._names[tid]

        def fetch(self, until_eof=False, **k):
            return iter(_read_records(self._path))

        def close(self):
            pass

    pysam.AlignmentFile = AlignmentFile
    sys.modules['pysam'] = pysam

    si = types.ModuleType('superintervals')
    si.IntervalMap = _IntervalMap
    sys.modules['superintervals'] = si

    skbio = types.ModuleType('skbio')
    skbio_al = types.ModuleType('skbio.alignment')

    class StripedSmithWaterman:  # pragma: no cover - never called on the clustering path
        def __init__(self, *a, **k):
            raise RuntimeError('skbio stand-in: not used on the clustering path')

    skbio_al.StripedSmithWaterman = StripedSmithWaterman
    skbio.alignment = skbio_al
    sys.modules['skbio'] = skbio
    sys.modules['skbio.alignment'] = skbio_al

    real_version = importlib.metadata.version

    def version(name):
        if name == 'fslr':
            return '0.3.10'
        return real_version(name)

    importlib.metadata.version = version


def load():
    """Return ``(cluster_module, main_module)`` of the reference."""
    if 'mods' in _loaded:
        return _loaded['mods']
    if not available():
        raise RuntimeError('reference not available')
    _install_stubs()
    if REF_ROOT not in sys.path:
        sys.path.insert(0, REF_ROOT)
    cluster = importlib.import_module('fslr.cluster')
    main = importlib.import_module('fslr.main')
    _loaded['mods'] = (cluster, main)
    return cluster, main


def run_cli(out_dir: str, name: str, extra_args=()):
    """Run the reference ``fslr --skip-alignment`` click command in-process."""
    from click.testing import CliRunner
    _, main = load()
    args = ['--name', name, '--out', out_dir, '--ref', 'unused.fa', '--primers', '21q1',
            '--skip-alignment'] + list(extra_args)
    res = CliRunner().invoke(main.pipeline, args, catch_exceptions=True)
    return res


def run_stages(bed_path: str, bam_path: str, overlap=0.8, cutoffs=(1, 1, 0.66, 0.66, 0.66, 0.5),
               qlen_diff=0.04, n_aln_diff=0.25, cluster_mask=('subtelomere',), edge_threshold=10,
               filter_false=False):
    """Run the reference clustering stages (main.py:209-244) and return intermediates."""
    import pandas as pd
    cluster, _ = load()
    bed = pd.read_csv(bed_path, sep='\t')
    mask = set()
    allowed = set(bed['chrom'])
    for item in cluster_mask:
        if item in allowed or item == 'subtelomere':
            mask.add(item)
    lengths = cluster.get_chromosome_lengths(bam_path)
    bed, chr_lengths, mask, cmap = cluster.rename_chromosomes(bed, lengths, mask)
    if filter_false:
        bed = cluster.delete_false(bed)
    fillings = cluster.keep_fillings(bed)
    data = cluster.prepare_data(fillings, mask, chr_lengths, threshold=500_000)
    tree = cluster.build_interval_trees(data)
    match_df, G = cluster.query_interval_trees(tree, data, overlap, list(cutoffs), edge_threshold,
                                               qlen_diff, n_aln_diff)
    subgraphs = cluster.get_subgraphs(G)
    return dict(bed=bed, fillings=fillings, data=data, match_df=match_df, G=G, subgraphs=subgraphs,
                chrom_map=cmap)
