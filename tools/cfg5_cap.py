#!/usr/bin/env python3
"""Config 5 (10M reads x 1-64 Zipf, seed 13) on one GPU: the edge cap's device replay.

Builds the input, runs the sweep query, then times fslr_apply_edge_cap (wall clock around the call,
which syncs) over --reps repetitions (each after a fresh query, so every replay starts from E*), and
checks the capped graph against the committed oracle results: the 50k-read sample
(tests/golden/cfg5/sample50k_capped.npz) and, when present, the full-graph digests
(tests/golden/cfg5/full_capped.json).  One JSON line on stdout; progress on stderr.

    python tools/cfg5_cap.py [--reps 3] > gpurun_out/cfg5_cap.json
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, 'tests', 'golden'))
GOLDEN = os.path.join(REPO, 'tests', 'golden', 'cfg5')


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--reps', type=int, default=3)
    args = ap.parse_args()
    import torch
    from fslr_amd import _lib, synth
    from fslr_amd.prep import fold_overlap_threshold, pass_table
    from make_cfg5_full import digests

    with open(os.path.join(GOLDEN, 'sample50k_capped.json')) as fh:
        meta = json.load(fh)
    t = time.perf_counter()
    s = synth.generate(meta['reads'], meta['lmax'], meta['seed'], dist=meta['dist'])
    csr = s.interval_data().csr()
    del s
    log(f'input {csr.n_reads} reads {csr.n_intervals} intervals in {time.perf_counter() - t:.0f}s')
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    ctx = _lib.Context(0, stream=stream.cuda_stream)
    ctx.load_csr(csr, fold_overlap_threshold(csr.iv_aln, 0.8))
    ctx.reserve_edges(12 * csr.n_reads)
    pt = pass_table([1, 1, 0.66, 0.66, 0.66, 0.5])
    out = {'reads': csr.n_reads, 'intervals': csr.n_intervals, 'rep_ms': [], 'query_ms': []}
    for rep in range(args.reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ctx.build_index()
        st = ctx.run_query(1 - 0.04, 1 - 0.25, pt, 10, engine='sweep')
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        cap = ctx.apply_edge_cap(10)
        t2 = time.perf_counter()
        out['query_ms'].append(round((t1 - t0) * 1e3, 2))
        out['rep_ms'].append(round((t2 - t1) * 1e3, 2))
        log(f'rep {rep}: index+query {out["query_ms"][-1]} ms, cap replay {out["rep_ms"][-1]} ms: {cap}')
    out['cap'] = cap
    out['e_star_edges'] = int(st['n_edges'])
    ne = ctx.stats()['n_edges']
    a, b, I, U = ctx.edges(ne)
    fwd = ctx.fwd_degree()
    ctx.components()
    lab = ctx.labels()
    S = meta['sample']
    z = np.load(os.path.join(GOLDEN, 'sample50k_capped.npz'))
    own = a < S
    got = sorted(zip(a[own].tolist(), b[own].tolist(), I[own].tolist(), U[own].tolist()))
    want = sorted(zip(z['a'].tolist(), z['b'].tolist(), z['I'].tolist(), z['U'].tolist()))
    out['sample_edges_equal'] = got == want
    out['sample_fwd_equal'] = bool(np.array_equal(fwd[:S], z['fwd']))
    d = digests(a, b, I, U, fwd, lab)
    out['digests'] = d
    full = os.path.join(GOLDEN, 'full_capped.json')
    if os.path.exists(full):
        with open(full) as fh:
            ref = json.load(fh)
        out['full_equal'] = {k: d[k] == ref[k] for k in ('edges_sha256', 'fwd_sha256', 'labels_sha256', 'n_edges',
                                                          'max_fwd')}
    print(json.dumps(out))


if __name__ == '__main__':
    main()
