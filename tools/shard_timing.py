#!/usr/bin/env python3
"""Per-rank device time of the multi-GPU step, measured on ONE GPU (no collective).

For world sizes W in --worlds, every shard r of W runs the rank's device work
(build_index for its shard, fslr_query_shard, local union-find) in its own
context, timed with HIP events over --steps repetitions; the merge that follows
the RCCL all-gather (W-1 label unions + finalize) is timed on stand-in labels.
Prints one JSON object: per W the max / mean over shards of each phase, the
label-merge time, and the single-GPU step for comparison.  The all-gather
itself needs W GPUs and is not measured here.

    python tools/shard_timing.py [--reads 1000000] [--worlds 1,2,4,8]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--reads', type=int, default=1_000_000)
    ap.add_argument('--lmax', type=int, default=16)
    ap.add_argument('--seed', type=int, default=11)
    ap.add_argument('--dist', default='uniform')
    ap.add_argument('--worlds', default='1,2,4,8')
    ap.add_argument('--steps', type=int, default=5)
    args = ap.parse_args()

    import torch
    from fslr_amd import _lib, synth
    from fslr_amd.prep import fold_overlap_threshold, pass_table

    s = synth.generate(args.reads, args.lmax, args.seed, dist=args.dist)
    csr = s.interval_data().csr()
    thr = fold_overlap_threshold(csr.iv_aln, 0.8)
    pt = pass_table([1, 1, 0.66, 0.66, 0.66, 0.5])
    qcut, ncut = 1 - 0.04, 1 - 0.25
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    n = csr.n_reads
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(5)]
    out = {'n_reads': n, 'n_intervals': int(csr.n_intervals), 'worlds': {}}
    print(f'input {n} reads, {csr.n_intervals} intervals', file=sys.stderr, flush=True)

    ctx = _lib.Context(0, stream=stream.cuda_stream)
    ctx.load_csr(csr, thr)
    ctx.reserve_edges(12 * n)
    for W in [int(x) for x in args.worlds.split(',')]:
        per = []
        for r in range(W):
            ctx.set_shard(r, W)
            t = np.zeros((args.steps, 4))
            for k in range(args.steps + 1):
                ev[0].record(stream)
                ctx.build_index()
                ev[1].record(stream)
                if W == 1:
                    ctx.query(qcut, ncut, pt, 10)
                else:
                    ctx.query_shard(qcut, ncut, pt, r, W)
                ev[2].record(stream)
                ctx.components()
                ev[3].record(stream)
                torch.cuda.synchronize()
                if k:
                    t[k - 1] = [ev[0].elapsed_time(ev[1]), ev[1].elapsed_time(ev[2]), ev[2].elapsed_time(ev[3]),
                                ev[0].elapsed_time(ev[3])]
            st = ctx.stats()
            per.append(dict(zip(('index_ms', 'query_ms', 'components_ms', 'total_ms'), np.median(t, 0).tolist()),
                            pairs=int(st['evaluated_pairs']), edges=int(st['n_edges'])))
            print(f'W={W} r={r} {per[-1]}', file=sys.stderr, flush=True)
        # merge after the all-gather: W-1 unions of N (k, label_g[k]) pairs + finalize
        merge_ms = 0.0
        if W > 1:
            lab = torch.from_numpy(ctx.labels().astype(np.int32)).to('cuda')
            g = lab.repeat(W)
            tm = []
            for k in range(args.steps + 1):
                ev[0].record(stream)
                ctx.union_pairs(None, g.data_ptr(), W * n, on_device=True)     # as DeviceShardMerge
                ctx.finalize_labels()
                ev[1].record(stream)
                torch.cuda.synchronize()
                if k:
                    tm.append(ev[0].elapsed_time(ev[1]))
            merge_ms = float(np.median(tm))
        agg = {k: {'max': max(p[k] for p in per), 'mean': float(np.mean([p[k] for p in per]))}
               for k in ('index_ms', 'query_ms', 'components_ms', 'total_ms')}
        agg['merge_ms'] = merge_ms
        agg['pairs_sum'] = sum(p['pairs'] for p in per)
        agg['per_shard'] = per
        out['worlds'][W] = agg
    one = out['worlds'].get(1)
    for W, a in out['worlds'].items():
        step = a['total_ms']['max'] + a['merge_ms']
        a['est_step_ms_excl_allgather'] = step
        if one:
            a['est_speedup_excl_allgather'] = one['total_ms']['max'] / step
    ctx.close()
    print(json.dumps(out))


if __name__ == '__main__':
    main()
