#!/usr/bin/env python3
"""Golden sample for BASELINE config 5 (10M reads, 1-64 fillings, truncated Zipf 1.5, seed 13).

The C oracle (oracle/fslr_oracle.c, pinned to the reference's own outputs by
tests/test_oracle_golden.py) runs the reference loop WITH the per-read edge cap
(cluster.py:223-224, search order of the superintervals stand-in) over query reads
[0, SAMPLE): the loops of those reads depend only on lower-rank reads, so their
edges and edges-per-loop are exactly those of the full run.  Saved as
tests/golden/cfg5/sample50k_capped.npz (+ .json stats).

    python tests/golden/make_cfg5_sample.py      (~10 min, ~20 GB RAM)
"""
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
from fslr_amd import synth  # noqa: E402
from oracle import oracle as O  # noqa: E402

READS, LMAX, SEED, SAMPLE = 10_000_000, 64, 13, 50_000


def main():
    t = time.perf_counter()
    s = synth.generate(READS, LMAX, SEED, dist='zipf')
    csr = s.interval_data().csr()
    del s
    print(f'CSR {csr.n_reads} reads {csr.n_intervals} intervals in {time.perf_counter() - t:.0f}s', flush=True)
    cnt = np.diff(csr.read_off)
    oc = O.OracleCSR(csr.read_off, csr.iv_chrom, csr.iv_start, csr.iv_end, csr.iv_aln,
                     np.repeat(csr.read_qlen2, cnt), np.repeat(csr.read_nal, cnt), csr.data_pos)
    t = time.perf_counter()
    o = O.run_core(oc, use_cap=True, query_end=SAMPLE)
    print(f'oracle sample in {time.perf_counter() - t:.0f}s: {o["stats"]}', flush=True)
    np.savez_compressed(os.path.join(HERE, 'cfg5', 'sample50k_capped.npz'), a=o['edge_a'].astype(np.int32),
                        b=o['edge_b'].astype(np.int32), I=o['edge_I'].astype(np.int16),
                        U=o['edge_U'].astype(np.int16), fwd=o['fwd'][:SAMPLE].astype(np.int16))
    meta = dict(o['stats'], reads=READS, lmax=LMAX, seed=SEED, dist='zipf', sample=SAMPLE, use_cap=True,
                n_intervals=csr.n_intervals, generator='tests/golden/make_cfg5_sample.py')
    with open(os.path.join(HERE, 'cfg5', 'sample50k_capped.json'), 'w') as fh:
        json.dump(meta, fh, indent=1)


if __name__ == '__main__':
    main()
