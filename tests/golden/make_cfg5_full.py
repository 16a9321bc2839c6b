#!/usr/bin/env python3
"""Full-graph digests for BASELINE config 5 (10M reads, 1-64 fillings, truncated Zipf 1.5, seed 13).

The C oracle (oracle/fslr_oracle.c, pinned to the reference's own outputs by
tests/test_oracle_golden.py) runs the reference loop WITH the per-read edge cap
(cluster.py:197-224, search order of the superintervals stand-in) over EVERY query
read, then components (cluster.py:230-234).  The graph is far too large to commit,
so only digests and counts are saved (tests/golden/cfg5/full_capped.json):

* ``edges_sha256``  sha256 of the capped edge list (a = the read whose loop formed the
  edge, b = its partner, I, U), rows sorted by (a, b), as little-endian int32 columns
  a | b | I | U concatenated;
* ``fwd_sha256``    sha256 of the edges formed per loop, int32[n_reads];
* ``labels_sha256`` sha256 of the min-rank component label of every read (a read
  without edges is its own label), int32[n_reads] — what ``fslr_get_labels`` returns;
* counts: edges, components, max forward degree, evaluated pairs.

``digests()`` is the one definition both this script and the GPU test use.

    python tests/golden/make_cfg5_full.py       (single-threaded oracle, ~1 h, ~30 GB RAM)
"""
import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

READS, LMAX, SEED = 10_000_000, 64, 13
OUT = os.path.join(HERE, 'cfg5', 'full_capped.json')


def _sha(*cols):
    h = hashlib.sha256()
    for c in cols:
        h.update(np.ascontiguousarray(c, dtype='<i4').tobytes())
    return h.hexdigest()


def digests(a, b, I, U, fwd, labels):
    """Digests of a capped graph: (a, b, I, U) edge columns, forward degrees, min-rank labels."""
    a = np.asarray(a, np.int64)
    b = np.asarray(b, np.int64)
    o = np.lexsort((b, a))
    return dict(edges_sha256=_sha(a[o], b[o], np.asarray(I)[o], np.asarray(U)[o]),
                fwd_sha256=_sha(fwd), labels_sha256=_sha(labels), n_edges=int(a.size),
                max_fwd=int(np.max(fwd)) if len(fwd) else 0)


def labels_from_comp(comp):
    """Oracle component index (-1 = no edge) -> min-rank label per read."""
    comp = np.asarray(comp, np.int64)
    n = comp.size
    lab = np.arange(n, dtype=np.int64)
    has = comp >= 0
    if has.any():
        first = np.full(int(comp.max()) + 1, n, np.int64)
        idx = np.nonzero(has)[0]
        np.minimum.at(first, comp[idx], idx)
        lab[idx] = first[comp[idx]]
    return lab.astype(np.int32)


def main():
    from fslr_amd import synth
    from oracle import oracle as O
    t = time.perf_counter()
    s = synth.generate(READS, LMAX, SEED, dist='zipf')
    csr = s.interval_data().csr()
    del s
    print(f'CSR {csr.n_reads} reads {csr.n_intervals} intervals in {time.perf_counter() - t:.0f}s', flush=True)
    cnt = np.diff(csr.read_off)
    oc = O.OracleCSR(csr.read_off, csr.iv_chrom, csr.iv_start, csr.iv_end, csr.iv_aln,
                     np.repeat(csr.read_qlen2, cnt), np.repeat(csr.read_nal, cnt), csr.data_pos)
    del csr
    t = time.perf_counter()
    o = O.run_core(oc, use_cap=True, lean=True)
    el = time.perf_counter() - t
    print(f'oracle full run in {el:.0f}s: {o["stats"]}', flush=True)
    d = digests(o['edge_a'], o['edge_b'], o['edge_I'], o['edge_U'], o['fwd'], labels_from_comp(o['comp']))
    meta = dict(d, reads=READS, lmax=LMAX, seed=SEED, dist='zipf', use_cap=True, edge_threshold=10,
                n_intervals=int(oc.start.size), n_components=int(o['stats']['n_components']),
                evaluated_pairs=int(o['stats']['evaluated_pairs']), oracle_seconds=round(el, 1),
                generator='tests/golden/make_cfg5_full.py')
    with open(OUT, 'w') as fh:
        json.dump(meta, fh, indent=1)
    print(json.dumps(meta, indent=1))


if __name__ == '__main__':
    main()
