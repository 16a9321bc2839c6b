#!/usr/bin/env python3
"""BASELINE config 5 workload on one GPU: 10M reads, 1-64 fillings (truncated Zipf 1.5, seed 13).

1. host prep (synthetic .mappings.bed columns -> prepared data -> CSR), with progress lines;
2. device step (build_index + pair kernels + union-find) timed over --steps, HBM-resident inputs;
3. parity on a bounded sample: the device restricted to query reads [0, --sample) against the C
   oracle on the same reads (index over all reads): identical edges (a, b, I, U), forward degrees
   and evaluated-pair / Jaccard-evaluation counts.

    python tools/cfg5_check.py [--reads 10000000] [--sample 200000] > gpurun_out/cfg5.json
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
    ap.add_argument('--reads', type=int, default=10_000_000)
    ap.add_argument('--lmax', type=int, default=64)
    ap.add_argument('--seed', type=int, default=13)
    ap.add_argument('--dist', default='zipf')
    ap.add_argument('--steps', type=int, default=5)
    ap.add_argument('--sample', type=int, default=200_000)
    ap.add_argument('--cap', action='store_true',
                    help='compare the capped graph (fslr_apply_edge_cap) with the oracle\'s reference loop')
    ap.add_argument('--oracle-npz', default=None,
                    help='saved oracle result for query reads [0, --sample) (edges a, b, I, U, fwd and the '
                         'stats in the file name\'s JSON twin); skips running the oracle here')
    args = ap.parse_args()
    import torch
    from fslr_amd import _lib, synth
    from fslr_amd.prep import fold_overlap_threshold, pass_table
    from oracle import oracle as O

    t = time.perf_counter()
    s = synth.generate(args.reads, args.lmax, args.seed, dist=args.dist)
    log(f'generated {s.n_rows} rows in {time.perf_counter() - t:.0f}s')
    t = time.perf_counter()
    data = s.interval_data()
    del s
    log(f'prepared {len(data)} intervals in {time.perf_counter() - t:.0f}s')
    t = time.perf_counter()
    csr = data.csr()
    t_csr = time.perf_counter() - t
    log(f'CSR {csr.n_reads} reads, {csr.n_intervals} intervals in {t_csr:.0f}s')
    L = np.diff(csr.read_off)

    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    ctx = _lib.Context(0, stream=stream.cuda_stream, profiling=True)
    thr = fold_overlap_threshold(csr.iv_aln, 0.8)
    t = time.perf_counter()
    ctx.load_csr(csr, thr)
    t_up = time.perf_counter() - t
    log(f'uploaded in {t_up:.1f}s')
    ctx.reserve_edges(12 * csr.n_reads)
    pt = pass_table([1, 1, 0.66, 0.66, 0.66, 0.5])
    qcut, ncut = 1 - 0.04, 1 - 0.25

    def step():
        ctx.build_index()
        ctx.query(qcut, ncut, pt, 10)
        ctx.components()

    step()
    st = ctx.stats(check=False)
    if st['n_edges'] > ctx.edge_capacity or st['deferred'] > st['deferred_capacity']:
        ctx.reserve_edges(st['n_edges'] + 4096)
        ctx.reserve_deferred(int(st["deferred"]) + 4096)
        step()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    ms = 1000 * (time.perf_counter() - t) / args.steps
    st = ctx.stats()
    tm = ctx.timings()
    log(f'device step {ms:.2f} ms, {st["evaluated_pairs"]} evaluated pairs, {st["n_edges"]} edges')
    log(json.dumps({'stats': {k: (v if isinstance(v, str) else int(v)) for k, v in st.items()}, 'timings': tm}))
    if args.sample <= 0:
        print(json.dumps({'ms_per_step': ms, 'stats': {k: (v if isinstance(v, str) else int(v)) for k, v in st.items()}, 'timings': tm}))
        return 0

    # the reference's edge cap on the full query (it binds at this density): replay cost
    ctx.build_index()
    gs = ctx.run_query(qcut, ncut, pt, 10)
    torch.cuda.synchronize()
    t = time.perf_counter()
    cap = ctx.apply_edge_cap(10)
    t_cap = time.perf_counter() - t
    log(f'edge cap replay {t_cap:.2f}s: {cap}')
    S = min(args.sample, csr.n_reads)
    if args.cap:
        # capped graph: the edges formed in the loops of reads [0, S) (oriented (former, partner))
        ne = ctx.stats()['n_edges']
        a, b, I, U = ctx.edges(ne)
        keep = a < S
        a, b, I, U = a[keep], b[keep], I[keep], U[keep]
        gfwd = ctx.fwd_degree()[:S]
    else:
        # parity on query reads [0, sample) of E*
        ctx.build_index()
        gs = ctx.run_query(qcut, ncut, pt, 10, 0, S)
        a, b, I, U = ctx.edges(gs['n_edges'])
        gfwd = ctx.fwd_degree()[:S]
    cnt = np.diff(csr.read_off)
    t = time.perf_counter()
    if args.oracle_npz:
        z = np.load(args.oracle_npz)
        with open(args.oracle_npz[:-4] + '.json') as fh:
            ost = json.load(fh)
        o = {'edge_a': z['a'], 'edge_b': z['b'], 'edge_I': z['I'], 'edge_U': z['U'], 'fwd': z['fwd'], 'stats': ost}
    else:
        oc = O.OracleCSR(csr.read_off, csr.iv_chrom, csr.iv_start, csr.iv_end, csr.iv_aln,
                         np.repeat(csr.read_qlen2, cnt), np.repeat(csr.read_nal, cnt), csr.data_pos)
        o = O.run_core(oc, use_cap=bool(args.cap), query_end=S)
    t_or = time.perf_counter() - t
    log(f'oracle sample in {t_or:.0f}s')
    ge = sorted(zip(a.tolist(), b.tolist(), I.tolist(), U.tolist()))
    oe = sorted(zip(o['edge_a'].tolist(), o['edge_b'].tolist(), o['edge_I'].tolist(), o['edge_U'].tolist()))
    parity = {
        'sample_query_reads': S,
        'edges_device': len(ge), 'edges_oracle': len(oe), 'edges_identical': ge == oe,
        'fwd_identical': bool(np.array_equal(gfwd, o['fwd'][:S])),
        'evaluated_pairs_device': int(gs['evaluated_pairs']), 'evaluated_pairs_oracle': int(o['stats']['evaluated_pairs']),
        'jaccard_evals_device': int(gs['jaccard_evals']), 'jaccard_evals_oracle': int(o['stats']['jaccard_evals']),
        'oracle_seconds': t_or, 'capped': bool(args.cap),
    }
    parity['all_identical'] = bool(parity['edges_identical'] and parity['fwd_identical'] and (args.cap or (
        parity['evaluated_pairs_device'] == parity['evaluated_pairs_oracle'] and
        parity['jaccard_evals_device'] == parity['jaccard_evals_oracle'])))
    out = {
        'workload': f'cfg5: {csr.n_reads} reads x 1-{args.lmax} fillings ({args.dist} 1.5), seed {args.seed}',
        'n_reads': csr.n_reads, 'n_intervals': csr.n_intervals, 'mean_L': float(L.mean()), 'max_L': int(L.max()),
        'ms_per_step': ms, 'evaluated_pairs_per_step': int(st['evaluated_pairs']),
        'evaluated_pairs_per_s': st['evaluated_pairs'] / (ms / 1000), 'edges': int(st['n_edges']),
        'max_fwd_degree': int(st['max_fwd']), 'overflow_candidates': int(st['overflow_candidates']),
        'deferred': int(st['deferred']), 'phase_ms_last_step': tm, 'host_csr_s': t_csr, 'upload_s': t_up,
        'edge_cap': cap, 'edge_cap_replay_s': t_cap,
        'parity_sample': parity,
    }
    print(json.dumps(out), flush=True)
    ctx.close()
    return 0 if parity['all_identical'] else 1


if __name__ == '__main__':
    sys.exit(main())
