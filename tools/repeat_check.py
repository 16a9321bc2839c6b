#!/usr/bin/env python3
"""Repeat the E* query and the capped replay on one input many times against the oracle and report
which stage differs when a run does not match (diagnostics for intermittent mismatches)."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, 'tests'), os.path.join(REPO, 'tests', 'golden')]
from host_pipeline import host_prepare  # noqa: E402
from test_gpu_parity import gpu_run, oracle_from_csr  # noqa: E402
from fslr_amd import _lib  # noqa: E402
from oracle import oracle as O  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else 'capbind_1500'
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
data, _, _ = host_prepare(name)
csr = data.csr()
oE = O.run_core(oracle_from_csr(csr), use_cap=False)
oC = O.run_core(oracle_from_csr(csr), use_cap=True)
eset = lambda a, b, I, U: set(zip(np.asarray(a).tolist(), np.asarray(b).tolist(), np.asarray(I).tolist(),
                                   np.asarray(U).tolist()))
wantE = eset(oE['edge_a'], oE['edge_b'], oE['edge_I'], oE['edge_U'])
wantC = eset(oC['edge_a'], oC['edge_b'], oC['edge_I'], oC['edge_U'])
bad = 0
for rep in range(reps):
    for mode in ('E', 'C', 'P'):
        if mode == 'P':      # the product path: build_interval_trees + query_interval_trees
            from fslr_amd import cluster
            tree = cluster.build_interval_trees(data)
            _, G = cluster.query_interval_trees(tree, data, 0.8, [1, 1, 0.66, 0.66, 0.66, 0.5], 10, 0.04, 0.25)
            st = G.stats
            E = O.run_core(oracle_from_csr(csr), use_cap=False)
            g = dict(a=G.edges_ab[0], b=G.edges_ab[1], I=None, U=None, fwd=G.fwd, labels=G.labels, stats=st)
            ea, eb = G.edges_ab
            dev = tree.ctx
            a2, b2, I2, U2 = dev.edges(len(ea))
            g['a'], g['b'], g['I'], g['U'] = a2, b2, I2, U2
            tree.ctx.close()
        else:
            ctx = _lib.Context(0)
            g = gpu_run(ctx, csr, cap=None if mode == 'E' else 10)
            ctx.close()
        got = eset(g['a'], g['b'], g['I'], g['U'])
        want, o = (wantE, oE) if mode == 'E' else (wantC, oC)
        fwd_bad = np.flatnonzero(g['fwd'] != o['fwd'])
        lab = g['labels']
        ok = got == want and fwd_bad.size == 0
        if not ok:
            bad += 1
            print(f'rep {rep} {mode}: edges {len(got)} vs {len(want)}; missing {sorted(want - got)[:6]} '
                  f'extra {sorted(got - want)[:6]}; fwd differs at {fwd_bad[:8].tolist()} '
                  f'(dev {g["fwd"][fwd_bad[:8]].tolist()} want {o["fwd"][fwd_bad[:8]].tolist()}) '
                  f'stats {g["stats"]}', flush=True)
        else:
            # edges right: check the labels (union-find) against the edges
            from fslr_amd.dist import union_find_labels
            ref = union_find_labels(csr.n_reads, g['a'], g['b'])
            if not np.array_equal(ref, lab):
                bad += 1
                d = np.flatnonzero(ref != lab)
                print(f'rep {rep} {mode}: edges ok, labels differ at {d[:8].tolist()}', flush=True)
print(f'{bad} bad of {3 * reps}')
