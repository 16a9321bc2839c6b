#!/usr/bin/env python3
"""Digests of the oracle's graph for BASELINE config 3/4's input (1M reads, 1-16 fillings, uniform,
seed 11): E* (no cap; the cap at 10 does not bind on this input, max forward degree 9) and the
reference loop with the per-read edge cap at 3 (cluster.py:197-224, binding), as
tests/golden/make_cfg5_full.py defines them.  tests/test_gpu_configs.py checks the product's W = 8
chromosome split on one GPU against both.

    python tests/golden/make_cfg4_1m.py          (single-threaded oracle, a few minutes)
"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, HERE)

from make_cfg5_full import digests, labels_from_comp  # noqa: E402

READS, LMAX, SEED = 1_000_000, 16, 11
OUT = os.path.join(HERE, 'cfg5', 'cfg4_1m.json')


def main():
    import numpy as np
    from fslr_amd import synth
    from oracle import oracle as O
    csr = synth.generate(READS, LMAX, SEED).interval_data().csr()
    cnt = np.diff(csr.read_off)
    oc = O.OracleCSR(csr.read_off, csr.iv_chrom, csr.iv_start, csr.iv_end, csr.iv_aln,
                     np.repeat(csr.read_qlen2, cnt), np.repeat(csr.read_nal, cnt), csr.data_pos)
    out = dict(reads=READS, lmax=LMAX, seed=SEED, dist='uniform', n_intervals=int(csr.n_intervals),
               generator='tests/golden/make_cfg4_1m.py')
    for key, cap, thr in (('estar', False, 10), ('capped10', True, 10), ('capped3', True, 3)):
        t = time.perf_counter()
        o = O.run_core(oc, edge_threshold=thr, use_cap=cap, lean=True)
        d = digests(o['edge_a'], o['edge_b'], o['edge_I'], o['edge_U'], o['fwd'], labels_from_comp(o['comp']))
        out[key] = dict(d, n_components=int(o['stats']['n_components']),
                        evaluated_pairs=int(o['stats']['evaluated_pairs']),
                        oracle_seconds=round(time.perf_counter() - t, 1))
        print(key, out[key], flush=True)
    with open(OUT, 'w') as fh:
        json.dump(out, fh, indent=1)


if __name__ == '__main__':
    main()
