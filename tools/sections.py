#!/usr/bin/env python3
"""Section cycle split of the pair kernel (FSLR_SECTION_PROF build, `make -C fslr_amd/csrc prof`).

    python tools/sections.py [--reads 1000000] [--lmax 16] [--dist uniform] [--reps 3]

Each wave sums s_memtime deltas per section (query.hip SEC_*); the split is the share of
the summed wave time, so memory waits land in the section that first uses the data.
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
os.environ.setdefault('FSLR_LIB', os.path.join(REPO, 'fslr_amd', 'libfslr_hip_prof.so'))

NAMES = ['read setup', 'next-chunk map + loads', 'hit + dedupe (load wait)', 'gate + deferred puts',
         'match list', 'next-read prefetch', 'greedy + edges', 'wave total']


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--reads', type=int, default=1_000_000)
    ap.add_argument('--lmax', type=int, default=16)
    ap.add_argument('--seed', type=int, default=11)
    ap.add_argument('--dist', default='uniform')
    ap.add_argument('--reps', type=int, default=3)
    args = ap.parse_args()
    import numpy as np
    from fslr_amd import _lib, synth
    from fslr_amd.prep import fold_overlap_threshold, pass_table
    csr = synth.generate(args.reads, args.lmax, args.seed, dist=args.dist).interval_data().csr()
    ctx = _lib.Context(0)
    ctx.load_csr(csr, fold_overlap_threshold(csr.iv_aln, 0.8))
    ctx.reserve_edges(12 * csr.n_reads)
    pt = pass_table([1, 1, 0.66, 0.66, 0.66, 0.5])
    acc = np.zeros(8)
    for _ in range(args.reps):
        ctx.build_index()
        ctx.query(1 - 0.04, 1 - 0.25, pt, 10, 0, csr.n_reads)
        ctx.sync()
        acc += ctx.counters(80)[48:56].astype(np.float64)
    tot = acc[7]
    out = {n: round(float(v / tot), 4) for n, v in zip(NAMES, acc)}
    out['unaccounted'] = round(float(1 - acc[:7].sum() / tot), 4)
    out['cycles_per_read_wave'] = float(tot / args.reps / csr.n_reads)
    print(json.dumps(out, indent=1))
    ctx.close()


if __name__ == '__main__':
    main()
