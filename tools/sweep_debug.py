#!/usr/bin/env python3
"""Sweep-engine diagnostics on a small synthetic input: both engines' stats and edge counts."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from fslr_amd import _lib, synth
from fslr_amd.prep import fold_overlap_threshold, pass_table
n, lmax, seed = (int(x) for x in (sys.argv[1:4] if len(sys.argv) > 3 else (3000, 16, 11)))
csr = synth.generate(n, lmax, seed).interval_data().csr()
ctx = _lib.Context(0)
ctx.load_csr(csr, fold_overlap_threshold(csr.iv_aln, 0.8))
ctx.reserve_edges(12 * csr.n_reads)
ctx.build_index()
for engine in ('walk', 'sweep'):
    st = ctx.run_query(0.96, 0.75, pass_table([1, 1, 0.66, 0.66, 0.66, 0.5]), engine=engine)
    print(engine, {k: st[k] for k in ('n_edges', 'candidates', 'pair_tests', 'match_entries', 'matched_pairs',
                                      'evaluated_pairs', 'jaccard_evals', 'max_fwd', 'overflow_flags')})
    print(' raw counters', ctx.counters(400)[[0, 16, 32, 33, 34, 38, 39, 336, 352]].tolist())
ctx.query(0.96, 0.75, pass_table([1, 1, 0.66, 0.66, 0.66, 0.5]), engine='walk')
wa = set(zip(*[x.tolist() for x in ctx.edges(ctx.stats()['n_edges'])]))
ctx.query(0.96, 0.75, pass_table([1, 1, 0.66, 0.66, 0.66, 0.5]), engine='sweep')
sw = set(zip(*[x.tolist() for x in ctx.edges(ctx.stats()['n_edges'])]))
L = np.diff(csr.read_off)
print('sweep subset of walk:', sw <= wa, 'extra', len(sw - wa), 'missing', len(wa - sw))
miss = sorted(wa - sw)[:15]
print('missing sample (a,b,I,U,LA,LB):', [(a, b, i, u, int(L[a]), int(L[b])) for a, b, i, u in miss])
print('present sample:', [(a, b, i, u, int(L[a]), int(L[b])) for a, b, i, u in sorted(sw)[:10]])
print('extra sample:', [(a, b, i, u, int(L[a]), int(L[b])) for a, b, i, u in sorted(sw - wa)[:10]])
