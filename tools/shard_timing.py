#!/usr/bin/env python3
"""Per-rank phase timing of the chromosome-split sweep, measured on ONE GPU.

For each world size W the ranks' work is run one rank at a time on cuda:0 with the data a rank
would hold (every read; the index of its own chromosomes):
  part[r]  = build_index (filtered) + fslr_sweep_partition (sweep, pack, route; ends in a sync)
  eval[d]  = fslr_sweep_evaluate (sort + pair kernel) over the entries destined to d, + its local
             forest (fslr_local_forest) and the copy of its (read, root) pairs for the exchange
  merge    = union-find over the W gathered forests' pairs (the replicated step)
and the single-context step (build_index + sweep query + components) as the W = 1 baseline.
The exchange itself cannot run on one GPU; it is priced from the bytes each rank moves
(entries all_to_all: the off-rank share of its entries; forest all_gather: 8 B x the largest
rank's pair count x (W - 1)) at an
assumed per-GPU xGMI rate (--xgmi-gbs, default 300 GB/s of the 7 x ~153 GB/s links, both
directions shared) plus a fixed per-collective latency (--coll-us).

    python tools/shard_timing.py --reads 1000000 --lmax 16 > gpurun_out/shard_cfg4.json
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--reads', type=int, default=1_000_000)
    ap.add_argument('--lmax', type=int, default=16)
    ap.add_argument('--dist', default='uniform')
    ap.add_argument('--seed', type=int, default=1)
    ap.add_argument('--worlds', default='1,2,4,8')
    ap.add_argument('--reps', type=int, default=5)
    ap.add_argument('--xgmi-gbs', type=float, default=300.0)
    ap.add_argument('--coll-us', type=float, default=30.0)
    ap.add_argument('--split', default='chrom', choices=['chrom', 'position'],
                    help='chrom: whole chromosomes per rank (chrom_owner); position: cost-balanced ranges of sorted '
                         'positions (position_plan), as SweepShard(split=...)')
    ap.add_argument('--plan-tests-only', action='store_true',
                    help='position split planned from pair tests and positions only (round-5 first version)')
    ap.add_argument('--chrom0-weight', type=float, default=0.0,
                    help='> 0: chromosome 0 gets this many times the number of chromosomes as its locus weight '
                         '(1.2: ~55 %% of the intervals on one chromosome, tests/test_dist.py skewed_case)')
    args = ap.parse_args()
    import torch
    from fslr_amd import _lib, synth
    from fslr_amd.dist import chrom_counts_of, chrom_owner, position_plan
    from fslr_amd.prep import fold_overlap_threshold, pass_table

    t = time.perf_counter()
    w = None
    if args.chrom0_weight > 0:
        w = np.ones(len(synth.CHROMS))
        w[0] = len(synth.CHROMS) * args.chrom0_weight
    s = synth.generate(args.reads, args.lmax, args.seed, dist=args.dist, chrom_weights=w)
    csr = s.interval_data().csr()
    del s
    log(f'data: {csr.n_reads} reads, {csr.n_intervals} intervals in {time.perf_counter() - t:.0f}s')
    n = csr.n_reads
    thr = fold_overlap_threshold(csr.iv_aln, 0.8)
    pt = pass_table([1, 1, 0.66, 0.66, 0.66, 0.5])
    qc, nc = 1 - 0.04, 1 - 0.25
    dev = torch.device('cuda', 0)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)

    def timed(fn, reps):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append(1000 * (time.perf_counter() - t0))
        return float(np.median(ts))

    # W = 1: the single-context step (the bench's step without the cap)
    c1 = _lib.Context(0, stream=stream.cuda_stream)
    c1.load_csr(csr, thr)
    c1.reserve_edges(12 * n)

    def single():
        c1.build_index()
        c1.query(qc, nc, pt, 10, engine='sweep')
        c1.components()
    t1 = timed(single, args.reps)
    st1 = c1.stats()
    c1_labels = c1.labels()
    log(f'W=1 step {t1:.3f} ms, {st1["n_edges"]} edges, {st1["match_entries"]} entries')
    c1.close()

    cp = _lib.Context(0, stream=stream.cuda_stream)
    cp.load_csr(csr, thr)
    ce = _lib.Context(0, stream=stream.cuda_stream)
    ce.load_csr(csr, thr)
    ce.reserve_edges(12 * n)
    counts = chrom_counts_of(csr)
    out = {'workload': f'{n} reads x 1-{args.lmax} ({args.dist}), seed {args.seed}'
                       + (f', chromosome 0 weight {args.chrom0_weight} x {len(counts)}' if w is not None else ''),
           'split': args.split, 'largest_chrom_share': float(counts.max() / counts.sum()), 'n_reads': n,
           'n_intervals': int(csr.n_intervals), 'single_step_ms': t1, 'match_entries': int(st1['match_entries']),
           'edges': int(st1['n_edges']), 'xgmi_gbs_assumed': args.xgmi_gbs, 'collective_latency_us': args.coll_us,
           'worlds': []}
    if args.split == 'position':
        cp.set_chrom_filter(None)
        cp.build_index()
        tile_tests, tile_reach = cp.position_costs()
        tile_entries = cp.position_entries(qc, nc, pt, 10)
    for W in [int(x) for x in args.worlds.split(',')]:
        owner = chrom_owner(counts, W)
        plan = (position_plan(tile_tests, tile_reach, int(csr.n_intervals), W,
                              tile_entries=None if args.plan_tests_only else tile_entries)
                if args.split == 'position' else None)
        part, part_rep, segs, sent = [], [], [[] for _ in range(W)], []
        index_ms, rank_tests, rank_pos, rank_entries = [], [], [], []
        buf = torch.empty(max(1 << 16, int(1.2 * st1['match_entries'] / W) + 4096), dtype=torch.int64, device=dev)
        for r in range(W):
            if plan is not None and W > 1:
                cp.set_position_filter(*plan[r])
            else:
                cp.set_chrom_filter(owner == r if W > 1 else None)
            res = {}

            def p():
                nonlocal buf
                cp.build_index()
                ok, cnt = cp.sweep_partition(qc, nc, pt, W, 6, buf)
                if not ok:
                    buf = torch.empty(int(cnt.sum() * 1.1) + 4096, dtype=torch.int64, device=dev)
                    ok, cnt = cp.sweep_partition(qc, nc, pt, W, 6, buf)
                res['cnt'] = cnt
            part.append(timed(p, args.reps))
            index_ms.append(timed(cp.build_index, args.reps))
            if plan is not None and W > 1:
                lo, hi, end = plan[r]
                rank_tests.append(int(tile_tests[lo // 64:(hi + 63) // 64].sum()))
                rank_entries.append(int(tile_entries[lo // 64:(hi + 63) // 64].sum()))
                rank_pos.append(int(hi - lo))
            cnt = res['cnt']
            if W > 1:
                # the repeat step's partition (SweepShard.step(repeat=True)): no readback inside
                def pr():
                    cp.build_index()
                    cp.sweep_partition_repeat(qc, nc, pt, W, 6, buf)
                part_rep.append(timed(pr, args.reps))
                assert not cp.stats()['overflow_flags'] & 32
            pos = np.concatenate([[0], np.cumsum(cnt)])
            for d in range(W):
                segs[d].append(buf[pos[d]:pos[d + 1]].clone())
            sent.append(cnt)
        evl, nedges, elists, npairs = [], [], [], []
        for d in range(W):
            ent = torch.cat(segs[d])
            ebuf = torch.empty(max(1, int(1.5 * st1['n_edges'] / W) + 4096), dtype=torch.int64, device=dev)

            def e():
                ce.sweep_evaluate(qc, nc, pt, ent, ent.numel())
                if W == 1:
                    ce.components()
                else:
                    ce.local_forest(count=False)               # the merge's (read, root) pairs
                    ce.forest_pairs_into(ebuf, ebuf.numel())
            evl.append(timed(e, args.reps))
            ne = ce.stats()['n_edges']
            nedges.append(ne)
            fp = ce.local_forest() if W > 1 else 0
            npairs.append(fp)
            elists.append(ebuf[:fp].clone())
            segs[d] = None
            del ent
        assert sum(nedges) == st1['n_edges'], (nedges, st1['n_edges'])
        m = max(1, max(npairs))
        gathered = torch.full((W * m,), -1, dtype=torch.int64, device=dev)
        for d in range(W):
            gathered[d * m:d * m + npairs[d]] = elists[d]
        merge = timed(lambda: ce.components_from_pairs(gathered, W * m), args.reps) if W > 1 else 0.0
        if W > 1:
            ref = c1_labels
            got = ce.labels()
            assert np.array_equal(got, ref), 'merged labels differ from the single context'
        sent = np.array(sent)
        off_rank = np.array([sent[r].sum() - sent[r, r] for r in range(W)])
        recv = sent.sum(axis=0)
        a2a_ms = 0.0 if W == 1 else (8 * max(off_rank.max(), (recv - np.diag(sent)).max()) / (args.xgmi_gbs * 1e6)
                                     + 2 * args.coll_us / 1000)
        gather_ms = 0.0 if W == 1 else 8 * m * (W - 1) / (args.xgmi_gbs * 1e6) + args.coll_us / 1000
        # + the all_reduce of (max forward degree, error flag, edge count) between evaluation and gather
        step = max(part) + a2a_ms + max(evl) + gather_ms + merge + (args.coll_us / 1000 if W > 1 else 0.0)
        # repeat steps: no count exchange and no all_reduce (one collective latency less in the a2a
        # model, none for the reduce), the partition without its readback
        step_rep = (max(part_rep) + a2a_ms - args.coll_us / 1000 + max(evl) + gather_ms + merge) if W > 1 else step
        row = {'W': W, 'part_ms': part, 'part_repeat_ms': part_rep, 'eval_ms': evl, 'merge_ms': merge,
               'part_max_over_mean': float(max(part) / np.mean(part)),
               'part_repeat_max_over_mean': float(max(part_rep) / np.mean(part_rep)) if part_rep else 1.0,
               'eval_max_over_mean': float(max(evl) / np.mean(evl)), 'plan': plan, 'index_ms': index_ms,
               'rank_tests': rank_tests, 'rank_positions': rank_pos, 'rank_entries_planned': rank_entries,
               'a2a_ms_model': a2a_ms, 'projected_step_repeat_ms': step_rep, 'projected_speedup_repeat': t1 / step_rep,
               'gather_ms_model': gather_ms, 'entries_sent_per_rank': sent.sum(axis=1).tolist(),
               'entries_recv_per_rank': recv.tolist(), 'edges_per_rank': nedges, 'forest_pairs_per_rank': npairs,
               'projected_step_ms': step,
               'projected_speedup': t1 / step}
        log(f'W={W}: part max {max(part):.3f} ms, eval max {max(evl):.3f} ms, merge {merge:.3f} ms, '
            f'a2a {a2a_ms:.3f} ms, gather {gather_ms:.3f} ms -> {step:.3f} ms ({t1 / step:.2f}x); repeat steps '
            f'{step_rep:.3f} ms ({t1 / step_rep:.2f}x)')
        out['worlds'].append(row)
        print(json.dumps(row), flush=True)
    print(json.dumps(out), flush=True)
    cp.close()
    ce.close()


if __name__ == '__main__':
    main()
