#!/usr/bin/env python3
"""Headline benchmark: evaluated Jaccard read-pair compares / s on the 1M-read interval cluster.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...      (one process per GPU, RCCL)

Workload (BASELINE.json configs[2]): 1,000,000 synthetic reads,
1-16 fillings each (seed 11), default clustering parameters.  Inputs are resident
in HBM before timing.  One step = the whole device hot path:
build_index (cluster.py:124) + pair kernel over this rank's query reads
(cluster.py:187-227) + union-find components (cluster.py:230) [+ RCCL label
exchange when N > 1].  ``value`` = evaluated read pairs of the whole job per
second (unit of work: a unique candidate pair whose predicate is evaluated,
SURVEY.md §8d).  Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK = 8.0e12          # MI355X_MICROARCH.md: HBM3E 8 TB/s spec
TRAFFIC_JSON = os.path.join(REPO, 'profiles', 'pmc_traffic_latest.json')


def kernel_source_hash():
    """sha256 of the pair-kernel sources: ties a committed PMC summary to the code it measured."""
    import hashlib
    h = hashlib.sha256()
    for f in ('query.hip', 'kernels.hpp'):
        with open(os.path.join(REPO, 'fslr_amd', 'csrc', f), 'rb') as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=10)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--reads', type=int, default=1_000_000)
    ap.add_argument('--lmax', type=int, default=16)
    ap.add_argument('--seed', type=int, default=11)
    ap.add_argument('--dist', default='uniform')
    ap.add_argument('--cpu-sample-reads', type=int, default=200_000,
                    help='query reads in the bounded CPU-oracle baseline sample (0 = skip)')
    ap.add_argument('--verify', action='store_true',
                    help='after timing, rank 0 checks its labels against a single-context run of all reads')
    ap.add_argument('--traffic-json', default=TRAFFIC_JSON,
                    help='rocprofv3 PMC summary (tools/pmc_traffic.py) giving HBM bytes per launch; used only '
                         'when it was measured on the current pair-kernel sources')
    return ap.parse_args()


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    args = parse()
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local_rank = int(os.environ.get('LOCAL_RANK', '0'))
    # FSLR_BENCH_DEVICE / FSLR_BENCH_BACKEND=gloo: rehearse N ranks on one GPU (tools/rehearse_multi.sh)
    dev_index = int(os.environ.get('FSLR_BENCH_DEVICE', local_rank))
    backend = os.environ.get('FSLR_BENCH_BACKEND', 'nccl')
    import torch
    torch.cuda.set_device(dev_index)
    dev = torch.device('cuda', dev_index)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if backend == 'nccl':
            dist.init_process_group('nccl', device_id=dev)      # RCCL over xGMI
        else:
            dist.init_process_group(backend)

    from fslr_amd import _lib, synth
    from fslr_amd.dist import DeviceShardMerge
    from fslr_amd.prep import fold_overlap_threshold, pass_table

    t0 = time.perf_counter()
    s = synth.generate(args.reads, args.lmax, args.seed, dist=args.dist)
    data = s.interval_data()
    csr = data.csr()
    log(f'[rank {rank}] input: {csr.n_reads} reads, {csr.n_intervals} intervals '
        f'(host prep {time.perf_counter() - t0:.1f}s)')

    # a dedicated (non-null) stream shared by the library, torch events and RCCL
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    ctx = _lib.Context(dev_index, stream=stream.cuda_stream, profiling=True)
    thr = fold_overlap_threshold(csr.iv_aln, 0.8)
    ctx.load_csr(csr, thr)
    ctx.reserve_edges(12 * csr.n_reads)
    pt = pass_table([1, 1, 0.66, 0.66, 0.66, 0.5])
    qcut, ncut = 1 - 0.04, 1 - 0.25
    merge = DeviceShardMerge(ctx, csr.n_reads, world, rank, dev) if world > 1 else None
    if world > 1:
        ctx.set_shard(rank, world)      # query-side index data (positions, ranges) for this shard's reads

    # pair-phase events per timed step (read after the timed region: no host sync between steps)
    ev_q = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            for _ in range(args.steps)]

    def step(k=None):
        ctx.build_index()
        if k is not None:
            ev_q[k][0].record(stream)
        if world > 1:
            ctx.query_shard(qcut, ncut, pt, rank, world)      # balanced rank blocks (fslr_query_shard)
        else:
            ctx.query(qcut, ncut, pt, 10)
        if k is not None:
            ev_q[k][1].record(stream)
        ctx.components()
        if merge is not None:
            merge()

    # warmup (also sizes the edge buffer)
    for w in range(max(1, args.warmup)):
        step()
        if w == 0:
            st = ctx.stats()
            if st['n_edges'] > ctx.edge_capacity:
                ctx.reserve_edges(st['n_edges'] + 4096)
    torch.cuda.synchronize()
    st = ctx.stats()

    # timed region
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for k in range(args.steps):
        step(k)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    st = ctx.stats()

    tot = torch.tensor([elapsed, float(st['evaluated_pairs']), float(st['algo_bytes']), float(st['n_edges']),
                        float(st['jaccard_evals'])], dtype=torch.float64,
                       device=dev if backend == 'nccl' else 'cpu')
    if dist:
        t_max = tot[:1].clone()
        dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
        sums = tot[1:].clone()
        dist.all_reduce(sums)
        elapsed = float(t_max.item())
        pairs, algo_bytes, n_edges, jacc = (float(x) for x in sums.tolist())
    else:
        pairs, algo_bytes, n_edges, jacc = (float(x) for x in tot[1:].tolist())
    lib_t = ctx.timings()                     # hipEvents of the last step (library side)
    ms_per_step = 1000.0 * elapsed / args.steps
    value = pairs / (elapsed / args.steps)
    kernel_ms = float(np.mean([a.elapsed_time(b) for a, b in ev_q]))
    # per-launch algorithmic bytes of this rank's pair kernel (SURVEY §8d B_pair summed over its pairs)
    achieved = st['algo_bytes'] / (kernel_ms / 1000.0)
    traffic = None
    traffic_src = None
    # the committed PMC summary is of the single-GPU launch (all query reads); a shard's launch moves less
    if world == 1 and args.traffic_json and os.path.exists(args.traffic_json):
        with open(args.traffic_json) as fh:
            tj = json.load(fh)
        if tj.get('source_hash') == kernel_source_hash():
            traffic = tj.get('query_kernel_hbm_bytes_per_launch')
            traffic_src = os.path.relpath(args.traffic_json, REPO)

    verified = None
    if args.verify and rank == 0:
        got = ctx.labels()
        ref = _lib.Context(dev_index)      # full, unsharded
        ref.load_csr(csr, thr)
        ref.reserve_edges(12 * csr.n_reads)
        ref.run(qcut, ncut, pt)
        verified = bool(np.array_equal(got, ref.labels()))
        ref.close()
        log(f'[rank 0] labels identical to a single-context run: {verified}')

    cpu = None
    if rank == 0 and world == 1 and args.cpu_sample_reads > 0:
        cpu = cpu_baseline(csr, args.cpu_sample_reads)

    if rank == 0:
        n = csr.n_reads
        out = {
            'metric': 'Jaccard pair-compares/sec + HBM GB/s vs roofline, 1M-read interval cluster',
            'value': value,
            'unit': 'evaluated read pairs/s',
            'n_gpus': world,
            'steps': args.steps,
            'warmup': args.warmup,
            'ms_per_step': ms_per_step,
            'higher_is_better': True,
            'scaling': 'strong',
            'vs_baseline': None,
            'dtype': 'int32',
            'data': 'synthetic (SURVEY §8d generator)',
            'config': {
                'workload': f'cfg3: {n} reads x 1-{args.lmax} fillings ({args.dist}), seed {args.seed}, '
                            'overlap 0.8, cutoffs 1,1,.66,.66,.66,.5, qlen-diff .04, n-aln-diff .25',
                'n_reads': n, 'n_intervals': csr.n_intervals,
                'evaluated_pairs_per_step': int(pairs), 'jaccard_evals_per_step': int(jacc),
                'edges': int(n_edges), 'max_fwd_degree': int(st['max_fwd']),
                'kernel_stats_rank0': {k: int(st[k]) for k in ('candidates', 'overflow_candidates', 'gather_pairs',
                                                               'match_entries', 'matched_pairs')},
                'dense_equivalent_pairs_per_s': (n * (n - 1) / 2) / (elapsed / args.steps),
                'parallelism': f'query-read shards x{world} (64-rank blocks round robin) + RCCL label all_gather'
                if world > 1 else 'single GPU',
            },
            'roofline': {
                'bound': 'hbm',
                'kernel': 'query_kernel',
                'achieved': achieved / 1e9,
                'peak': HBM_PEAK / 1e9,
                'unit': 'GB/s',
                'frac': achieved / HBM_PEAK,
                'traffic': traffic,
                'traffic_source': traffic_src,
                'kernel_ms': kernel_ms,
                'algo_bytes_per_launch': int(st['algo_bytes']),
                'phase_ms_last_step': lib_t,
            },
            'cpu_baseline': cpu,
        }
        if verified is not None:
            out['verified_labels_vs_single_context'] = verified
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()
    ctx.close()


def cpu_baseline(csr, sample_reads):
    """Bounded CPU-oracle sample (oracle/fslr_oracle.c, 1 thread): query reads [0, sample)
    against all reads, index build included; evaluated pairs / s."""
    try:
        from oracle import oracle as O
    except Exception as e:  # pragma: no cover
        return {'error': f'oracle unavailable: {e}'}
    cnt = np.diff(csr.read_off)
    oc = O.OracleCSR(csr.read_off, csr.iv_chrom, csr.iv_start, csr.iv_end, csr.iv_aln,
                     np.repeat(csr.read_qlen2, cnt), np.repeat(csr.read_nal, cnt), csr.data_pos)
    sample = min(sample_reads, csr.n_reads)
    t = time.perf_counter()
    r = O.run_core(oc, use_cap=True, query_end=sample)
    dt = time.perf_counter() - t
    return {'value': r['stats']['evaluated_pairs'] / dt, 'unit': 'evaluated read pairs/s', 'cores': 1,
            'kind': 'port', 'seconds': dt,
            'sample': f'oracle/fslr_oracle.c on query reads [0, {sample}) of the same 1M-read input '
                      f'({r["stats"]["evaluated_pairs"]} evaluated pairs, index over all reads)'}


if __name__ == '__main__':
    main()
