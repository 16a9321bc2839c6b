"""Import the *reference* fslr (read-only at /root/reference) for golden-vector capture.

Test infrastructure only: used by ``make_golden.py`` and by the optional live
cross-check in ``tests/test_oracle_live.py``.  It never travels to the GPU box
(``/root/reference`` does not exist there) and nothing in the product imports it.

The reference imports packages that are not installed in this image
(SURVEY.md §8c): ``pysam``, ``superintervals`` (>= 0.2.10, unpinned, C++/Cython),
``skbio``.  They are replaced by stand-ins that restate only what the clustering
path needs:

* ``pysam.AlignmentFile(bam).lengths / .get_reference_name(tid)`` — the BAM
  header dictionary (``cluster.py:173-175``), decoded by ``fslr_amd.bam_header``.
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


def _install_stubs():
    from fslr_amd import bam_header

    pysam = types.ModuleType('pysam')

    class AlignmentFile:
        def __init__(self, path, mode='rb', *a, **k):
            refs = bam_header.read_bam_references(path)
            self._names = [n for n, _ in refs]
            self.lengths = tuple(l for _, l in refs)
            self.references = tuple(self._names)

        def get_reference_name(self, tid):
            return self._names[tid]

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
