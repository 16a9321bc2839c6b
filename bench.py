#!/usr/bin/env python3
"""Headline benchmark: Jaccard-evaluated read pairs / s on the 1M-read interval cluster.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...      (one process per GPU, RCCL)

Workload (BASELINE.json configs[2]): 1,000,000 synthetic reads,
1-16 fillings each (seed 11), default clustering parameters.  Inputs are resident
in HBM before timing.  One step = the whole device hot path: build_index
(cluster.py:124) + pair kernels over this rank's query reads (cluster.py:187-222)
+ the edge-cap check/replay (cluster.py:223-224; one rank) + union-find components
(cluster.py:230) [+ RCCL label exchange when N > 1].

``value`` = read pairs whose full predicate is evaluated (the length gate passes and
overall_jaccard_similarity runs: the unit SURVEY.md §8d defines and the reference's
measured 2.27e4 pairs/s counts) of the whole job per second.  Candidate
pairs (gate-rejected ones included) and the dense-equivalent rate are secondary fields.

``roofline``: the longest kernel of the step (HIP-event means over the timed steps), the
others in ``roofline_other_kernels``.  Sweep engine (default): the position sweep
k_sweep<2> — every sorted position's index record, gate word and forward
count and its read's gate ranges read once (48 B), plus each match entry written (8 B) —
and the pair stage k_sweep_pairs — each grouped match entry read once (8 B), each edge written
(10 B) and its union-find pre-hook (an atomicMin on the upper read's parent: 4 B read + 4 B
written), each read's forward degree written (4 B) (the same bytes for the fused variant
k_bucket_pairs, FSLR_PAIR_STAGE=fused, which reads the entries from the grouping's pass-1 buckets).  Walk engine: query_kernel, every
walked index record (16-B record + 8-B gate word) read once, each query read's header,
gate bounds and forward degree, each of its intervals' sorted position, row and scan
range, and the edge / deferred-list output.  ``achieved`` = those bytes ÷ the mean
duration of the timed launches, measured with hipEvents the library records around
each of those launches on its stream (fslr_get_stage_kernel_times).  ``traffic`` = HBM
bytes per launch from rocprofv3 PMC counters (tools/pmc_traffic.py), used only when that
summary was measured on the current sources of that kernel.

Prints ONE JSON line on rank 0.
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
# walk engine: bytes per walked record / per query read / per query interval / per edge / per deferred entry
B_WALK, B_READ, B_IVL, B_EDGE, B_DEFER = 24, 8 + 16 + 4, 4 + 12 + 8, 8 + 2, 8
# sweep engine: bytes per sorted position (record, gate word, forward count, read gate ranges) / per entry
B_POS, B_ENT = 16 + 8 + 8 + 16, 8
KERNEL_SOURCES = {'sweep': ('sweep.hip', 'wave.hpp', 'kernels.hpp'), 'walk': ('query.hip', 'kernels.hpp')}
KERNEL_NAME = {'sweep': 'k_sweep<2>', 'walk': 'query_kernel<0, false>'}
# the sweep's pair-stage kernel (the one fslr_get_stage_kernel_times(1) times): k_sweep_pairs over the
# grouped entries, or with FSLR_PAIR_STAGE=fused the bucket kernel fused with the grouping's pass 2
PAIR_STAGE = 'k_bucket_pairs' if os.environ.get('FSLR_PAIR_STAGE') == 'fused' else 'k_sweep_pairs'
# the reference's own rate on this config: 33,020,021 Jaccard-evaluated
# pairs in 1454.0 s of query_interval_trees, 1 core of the survey container, pure Python
REFERENCE_PY = {'value': 33_020_021 / 1454.0, 'unit': 'Jaccard-evaluated read pairs/s', 'cores': 1,
                'kind': 'reference', 'where': 'survey container (8-vCPU Xeon), not the GPU box',
                'sample': 'reference cluster.py, 1M reads x 1-16, query_interval_trees stage (BASELINE.md)'}


def kernel_source_hash(engine='sweep'):
    """sha256 of the dominant kernel's sources: ties a committed PMC summary to the code it measured."""
    import hashlib
    h = hashlib.sha256()
    for f in KERNEL_SOURCES[engine]:
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
    ap.add_argument('--engine', default='auto', choices=['auto', 'walk', 'sweep'],
                    help='pair engine of the timed step (fslr_hip.h FSLR_ENGINE_*); the walk engine always runs '
                         'once before timing to count the Jaccard-evaluated pairs of the input')
    ap.add_argument('--sync-cap', action='store_true',
                    help='check the edge cap with a host read in every timed step (default: on the device, '
                         'read once after the timed steps; a step that needed the replay reruns them this way)')
    ap.add_argument('--cpu-sample-stride', type=int, default=16,
                    help='single-thread CPU baseline: query reads of every k-th 64-rank block (0 = skip the '
                         'CPU baseline)')
    ap.add_argument('--cpu-threads', type=int, default=0,
                    help='threads of the all-core CPU baseline (0 = the affinity set, limited by OMP_NUM_THREADS)')
    ap.add_argument('--verify', action='store_true',
                    help='after timing, rank 0 checks its labels against a single-context run of all reads')
    ap.add_argument('--traffic-json', default=TRAFFIC_JSON,
                    help='rocprofv3 PMC summary (tools/pmc_traffic.py) giving HBM bytes per launch; used only '
                         'when it was measured on the current pair-kernel sources')
    return ap.parse_args()


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_share():
    """Threads of the all-core CPU baseline: every CPU in this process's affinity set (all
    host cores); OMP_NUM_THREADS (16 on the GPU box, its CPU share per GPU) gives the second point."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, 'sched_getaffinity') else (os.cpu_count() or 1)
    return max(1, n)


def cpu_policy():
    aff = len(os.sched_getaffinity(0)) if hasattr(os, 'sched_getaffinity') else None
    return (f'threads = the affinity set ({aff} CPUs); second point at OMP_NUM_THREADS='
            f'{os.environ.get("OMP_NUM_THREADS", "unset")} (16 when unset); {os.cpu_count()} CPUs visible on the host')


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
    from fslr_amd.dist import SweepShard, chrom_counts_of, chrom_owner, shard_range
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
    t_up = time.perf_counter()
    ctx.load_csr(csr, thr)                 # host packing + H2D of the CSR (synchronous)
    upload_s = time.perf_counter() - t_up
    h2d_bytes = 16 * csr.n_reads + csr.n_intervals * (16 + 4 + 4 + 16 + 8)
    ctx.reserve_edges(12 * csr.n_reads)
    pt = pass_table([1, 1, 0.66, 0.66, 0.66, 0.5])
    qcut, ncut = 1 - 0.04, 1 - 0.25
    # the input's unit count: the walk engine dedupes partners (the reference's seen-set) and counts
    # the pairs whose predicate is evaluated; the sweep evaluates the same pairs without counting them.
    # With N ranks each counts the pairs whose first read lies in its contiguous range (summed below).
    a0, a1 = shard_range(csr.n_reads, rank, world)
    ctx.build_index()
    counted = ctx.run_query(qcut, ncut, pt, 10, a0, a1, engine='walk')
    if world == 1:
        walk_edges = sorted(zip(*[x.tolist() for x in ctx.edges(counted['n_edges'])]))
        walk_fwd = ctx.fwd_degree()
    shard = None
    if world > 1:
        # chromosome-split sweep: this rank indexes and sweeps its chromosomes, routes
        # the match entries to the first read's owner (RCCL all_to_all), evaluates, merges labels
        shard = SweepShard(ctx, csr.n_reads, chrom_counts_of(csr), world, rank, dev, split='auto')

    def step(collect=False, repeat=False):
        if shard is not None:
            return shard.step(qcut, ncut, pt, 10, collect=collect, repeat=repeat)
        ctx.build_index()
        ctx.query(qcut, ncut, pt, 10, engine=args.engine)
        ctx.components()
        # cluster.py:223-224: the edge cap (one counter read; a replay + new components only if it binds).
        # A repeated step checks on the device without waiting for the host (the sticky word is read
        # after the timed steps; a step that needed the replay makes them rerun synchronously)
        if repeat and not args.sync_cap:
            ctx.edge_cap_deferred(10)
            return None
        if ctx.apply_edge_cap(10)['applied']:
            ctx.components()
        return None

    # warmup (also sizes the edge buffer); the last one reads the sweep's counters (multi-GPU)
    info = None
    for w in range(max(1, args.warmup)):
        info = step(collect=(w == max(1, args.warmup) - 1))
        if w == 0 and shard is None:
            st = ctx.stats(check=False)
            if st['n_edges'] > ctx.edge_capacity:
                ctx.reserve_edges(st['n_edges'] + 4096)
    torch.cuda.synchronize()
    st = ctx.stats()
    engine = st['engine']
    if world == 1 and engine != 'walk':
        ctx.query(qcut, ncut, pt, 10, engine=args.engine)
        se = ctx.stats()
        same = (sorted(zip(*[x.tolist() for x in ctx.edges(se['n_edges'])])) == walk_edges and
                bool(np.array_equal(ctx.fwd_degree(), walk_fwd)))
        if not same and not os.environ.get('FSLR_ABLATE'):           # profiling ablations only
            raise SystemExit(f'{engine} engine differs from the walk engine on this input')
        log(f'[rank 0] {engine} engine: edges and forward degrees identical to the walk engine')

    # timed regions: only the pair kernels' own events stay on the stream (profiling level 2); the
    # per-phase events are recorded in one extra untimed step afterwards.
    # 1. repeat steps (secondary): a query on unchanged input keeps its length-gate ranges and its entry
    #    count on the device (no mid-step readback), the edge cap checked on the device.
    # 2. full-work steps (`value`): every query recomputes the gate ranges (k_len_bounds) and, on one GPU,
    #    reads its entry count back and checks the cap with a host read, as a single query on new input
    #    does; with N ranks each step still skips the host round trips (the partition's counts are checked
    #    on the device against the synchronous step's), every kernel runs.
    ctx.set_profiling(2)

    def timed(repeat, reuse):
        ctx.set_query_reuse(reuse)
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        t0_ = time.perf_counter()
        for _ in range(args.steps):
            step(repeat=repeat)
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        return time.perf_counter() - t0_

    elapsed_rep = timed(True, True)
    if shard is None and not args.sync_cap and ctx.edge_cap_deferred_read():
        # a timed step's cap check fired: those steps needed the replay; time them synchronously
        log('[rank 0] the edge cap bound in a timed step: timing synchronous steps instead')
        args.sync_cap = True
        elapsed_rep = timed(True, True)
    elapsed = timed(shard is not None, False)        # one GPU: full synchronous steps
    ctx.set_query_reuse(True)
    if shard is not None:
        # the timed steps repeated the last warmup step without host syncs (SweepShard.step repeat):
        # every rank's device checks and edge counts must agree with it
        shard.verify_repeat()
    st = ctx.stats()
    kern = ctx.pair_kernel_times(args.steps)       # the full-work steps' main pair-kernel launches
    kern2 = ctx.stage_kernel_times(1, args.steps) if st['engine'] == 'sweep' else np.zeros(0)   # pair stage
    lib_t = None
    cold_ms = None
    if world == 1:
        ctx.set_profiling(1)
        step()
        torch.cuda.synchronize()
        lib_t = ctx.timings()                         # hipEvents of one untimed step (library side)
        # one cold step: a new input generation (fslr_set_thresholds), as the CLI's single query
        ctx.set_profiling(0)
        ctx.set_thresholds(thr)
        torch.cuda.synchronize()
        t = time.perf_counter()
        step()
        torch.cuda.synchronize()
        cold_ms = 1000.0 * (time.perf_counter() - t)

    sw = info['sweep_stats'] if info is not None else st          # this rank's sweep counters
    if world > 1:
        own_chroms = chrom_owner(chrom_counts_of(csr), world) == rank
        n_pos = int(chrom_counts_of(csr)[own_chroms].sum())          # positions of this rank's index
    else:
        n_pos = csr.n_intervals
    if st['engine'] == 'sweep':
        algo_bytes = B_POS * n_pos + B_ENT * sw['match_entries']
        algo_model = (f'{B_POS} B x sorted positions ({n_pos}: record, gate word, forward count, read gate '
                      f'ranges) + {B_ENT} B x match entries written ({sw["match_entries"]})')
    else:
        own = np.ones(csr.n_reads, bool)
        q_reads = int(own.sum())
        q_ivls = int(np.diff(csr.read_off)[own].sum())
        algo_bytes = (B_WALK * st['walked_records'] + B_READ * q_reads + B_IVL * q_ivls + B_EDGE * st['n_edges'] +
                      B_DEFER * st['deferred'])
        algo_model = (f'{B_WALK} B x walked records ({st["walked_records"]}) + {B_READ} B x query reads + {B_IVL} B x '
                      'query intervals + {B_EDGE} B x edges + {B_DEFER} B x deferred entries')
    cs = counted                                      # the walk engine's counts of this rank's read range
    tot = torch.tensor([elapsed, float(cs['evaluated_pairs']), float(cs['jaccard_evals']), float(st['n_edges']),
                        float(st['max_fwd']), elapsed_rep, float(st['matched_pairs'])], dtype=torch.float64,
                       device=dev if backend == 'nccl' else 'cpu')
    capped = bool(info['capped']) if info is not None else False
    if dist:
        t_max = tot[[0, 4, 5]].clone()
        dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
        sums = tot[[1, 2, 3, 6]].clone()
        dist.all_reduce(sums)
        elapsed, max_fwd, elapsed_rep = (float(x) for x in t_max.tolist())
        max_fwd = int(max_fwd)
        pairs, jacc, n_edges, matched = (float(x) for x in sums.tolist())
    else:
        pairs, jacc, n_edges, matched = (float(x) for x in tot[[1, 2, 3, 6]].tolist())
        max_fwd = int(st['max_fwd'])
    ms_per_step = 1000.0 * elapsed / args.steps
    value = jacc / (elapsed / args.steps)
    # the committed PMC summaries (profiles/pmc_traffic_latest.json, keyed by kernel) are of the
    # single-GPU launch on these sources; a shard's launch moves less
    tj = {}
    if world == 1 and args.traffic_json and os.path.exists(args.traffic_json):
        with open(args.traffic_json) as fh:
            tj = json.load(fh)
        if 'kernel' in tj:
            tj = {tj['kernel']: tj}
    src_hash = kernel_source_hash(st['engine'])

    def roofline(name, times, algo, model):
        kms = float(np.mean(times)) if times.size else float('nan')
        ach = algo / (kms / 1000.0)
        e = tj.get(name, {})
        traffic = e.get('hbm_bytes_per_launch') if e.get('source_hash') == src_hash else None
        valu = e.get('valu_issue_frac') if e.get('source_hash') == src_hash else None
        split = e.get('wave_cycle_split') if e.get('source_hash') == src_hash else None
        return {'bound': 'hbm', 'kernel': name, 'achieved': ach / 1e9, 'peak': HBM_PEAK / 1e9, 'unit': 'GB/s',
                'frac': ach / HBM_PEAK, 'traffic': traffic,
                # the roofline is HBM's (integer work, no MFMA); what limits these kernels is latency and
                # issue, not bytes: valu_issue_frac and wave_cycle_split say how far from the issue side
                'limiter': 'latency / issue (dependent LDS and gather chains), not HBM bytes: see valu_issue_frac, '
                           'wave_cycle_split',
                # the issue side beside the HBM side: 2 cycles per wave64 VALU instruction over the
                # launch's cycles on 1024 SIMDs (PMC), and where the wave-cycles went
                'valu_issue_frac': valu, 'wave_cycle_split': split,
                'traffic_source': os.path.relpath(args.traffic_json, REPO) if traffic else None,
                'traffic_basis': e.get('correction') if traffic else None,
                'waste_ratio': (traffic / algo) if traffic else None, 'kernel_ms': kms,
                'kernel_launches_timed': int(times.size), 'algo_bytes_per_launch': int(algo),
                'algo_bytes_model': model}

    roofs = [roofline(KERNEL_NAME[st['engine']], kern, algo_bytes, algo_model)]
    if kern2.size:
        # the pair stage: every grouped match entry read once (8 B), each edge written (a, b + I | U:
        # 10 B) and hooked into the union-find (atomicMin on parent[b]: 4 B read + 4 B written, the work
        # k_uf_hook_min did before round 6), each read's forward degree written (4 B); the 1-byte read
        # lengths it looks up stay in L2
        pb = B_ENT * sw['match_entries'] + (10 + 8) * st['n_edges'] + 4 * csr.n_reads
        roofs.append(roofline(PAIR_STAGE, kern2, pb,
                              f'{B_ENT} B x grouped match entries read ({sw["match_entries"]}) '
                              f'+ 10 B x edges written ({st["n_edges"]}) + 8 B x their union-find pre-hook '
                              f'(atomicMin on parent[b]) + 4 B x forward degrees ({csr.n_reads})'))
    # the headline roofline is the longest kernel's (HIP events over the timed steps)
    roofs.sort(key=lambda r: -r['kernel_ms'] if r['kernel_ms'] == r['kernel_ms'] else 0.0)
    head_roof = dict(roofs[0], phase_ms_last_step=lib_t,
                     selection='the longest kernel of the step by its HIP-event mean over the timed steps')
    # transfers around the device path (not in `value`): CSR upload before, labels / edges after
    t = time.perf_counter()
    labels = shard.labels() if shard is not None else ctx.labels()
    d2h_labels_s = time.perf_counter() - t
    t = time.perf_counter()
    ctx.edges(st['n_edges'])
    d2h_edges_s = time.perf_counter() - t
    transfer = {
        'upload_csr_s': upload_s, 'upload_csr_bytes': h2d_bytes,
        'd2h_labels_s': d2h_labels_s, 'd2h_edges_s': d2h_edges_s,
        'pcie_inclusive_value': jacc / (elapsed / args.steps + upload_s + d2h_labels_s + d2h_edges_s),
        'note': 'upload = host packing/validation + H2D of the CSR and data-order records, once per input; '
                'the step keeps inputs resident in HBM',
    }

    verified = None
    if args.verify and rank == 0:
        ref = _lib.Context(dev_index)      # full, unsharded
        ref.load_csr(csr, thr)
        ref.reserve_edges(12 * csr.n_reads)
        ref.run(qcut, ncut, pt)
        verified = bool(np.array_equal(labels, ref.labels()))
        ref.close()
        log(f'[rank 0] labels identical to a single-context run: {verified}')

    cpu = None
    if rank == 0 and world == 1 and args.cpu_sample_stride > 0:
        cpu = cpu_baseline(csr, args.cpu_sample_stride, args.cpu_threads or cpu_share(), int(jacc))

    if rank == 0:
        n = csr.n_reads
        out = {
            'metric': 'Jaccard pair-compares/sec + HBM GB/s vs roofline, 1M-read interval cluster',
            'value': value,
            'unit': 'Jaccard-evaluated read pairs/s',
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
                'jaccard_evals_per_step': int(jacc),
                'step': ('full work: index build, every pair kernel with the length-gate ranges recomputed, '
                         + ('the entry count read back mid-query, components and the edge-cap check by a host '
                            'read' if world == 1 else
                            'both RCCL exchanges, the forest merge; the partition counts checked on the device')),
                'kernel_evaluated_pairs_per_step': int(matched),
                'kernel_evaluated_pairs_per_s': matched / (elapsed / args.steps),
                'kernel_evaluated_note': 'read pairs the sweep actually evaluates (>= 1 match entry: first-fit, '
                                         'U, the cut); the other Jaccard-evaluated pairs have I = 0 and are '
                                         'decided without a kernel touching them (DESIGN.md §3.6)',
                'repeat_step_ms': 1000.0 * elapsed_rep / args.steps,
                'repeat_value': jacc / (elapsed_rep / args.steps),
                'repeat_note': 'the same step repeated on unchanged input: the length-gate ranges and the entry '
                               'count stay on the device, the edge cap is checked on the device',
                'candidate_pairs_per_step': int(pairs),
                'candidate_pairs_per_s': pairs / (elapsed / args.steps),
                'edges': int(n_edges), 'max_fwd_degree': max_fwd,
                'engine': st['engine'],
                'kernel_stats_rank0': {k: int(sw[k]) for k in ('candidates', 'walked_records', 'overflow_candidates',
                                                               'gather_pairs', 'match_entries', 'matched_pairs',
                                                               'deferred', 'pair_tests')},
                'interval_pair_tests_per_s_rank0': sw['pair_tests'] / (elapsed / args.steps)
                if st['engine'] == 'sweep' else None,
                'unit_count_source': 'walk engine run on the same input before timing (its seen-set counts the '
                                     'pairs whose predicate is evaluated; the sweep decides the same pairs, '
                                     'DESIGN.md §4)' + ('' if world == 1 else
                                                        '; each rank counts the pairs whose first read lies in '
                                                        'its contiguous read range, summed'),
                'edge_cap_bound': capped,
                'dense_equivalent_pairs_per_s': (n * (n - 1) / 2) / (elapsed / args.steps),
                'parallelism': (f'{shard.split}-split sweep x{world}: each rank indexes and sweeps '
                                + ('a cost-balanced range of the sorted positions (tests, positions, entries)'
                                   if shard.split == 'position' else 'its chromosomes')
                                + ', RCCL all_to_all of match entries to the first read\'s owner (64-rank blocks '
                                  'round robin), evaluation there, RCCL all_gather of local forests + union')
                if world > 1 else 'single GPU',
                'transfer': transfer,
                'cold_step_ms': cold_ms,
                'cold_step_note': 'one step after a new input generation (fslr_set_thresholds), timed alone: '
                                  'the same work as a timed full step',
            },
            'roofline': head_roof,
            'roofline_other_kernels': roofs[1:],
            'cpu_baseline': cpu,
        }
        if verified is not None:
            out['verified_labels_vs_single_context'] = verified
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()
    ctx.close()


def cpu_baseline(csr, stride, threads, gpu_jacc):
    """The C restatement (oracle/fslr_oracle.c) on the box's host cores, same input and unit:
    1 thread on the query reads of every ``stride``-th 64-rank block, then ``threads`` threads
    sharing one index over all query reads (E*; the cap does not bind on this input)."""
    try:
        from oracle import oracle as O
    except Exception as e:  # pragma: no cover
        return {'error': f'oracle unavailable: {e}'}
    cnt = np.diff(csr.read_off)
    oc = O.OracleCSR(csr.read_off, csr.iv_chrom, csr.iv_start, csr.iv_end, csr.iv_aln,
                     np.repeat(csr.read_qlen2, cnt), np.repeat(csr.read_nal, cnt), csr.data_pos)
    t = time.perf_counter()
    one = O.count_threads(oc, nthreads=1, stride=stride)
    dt1 = time.perf_counter() - t
    t = time.perf_counter()
    allc = O.count_threads(oc, nthreads=threads, stride=1)
    dta = time.perf_counter() - t
    env = os.environ.get('OMP_NUM_THREADS')
    t2 = int(env) if env and env.isdigit() else 16
    second = None
    if t2 != threads:
        t = time.perf_counter()
        c2 = O.count_threads(oc, nthreads=t2, stride=1)
        dt2 = time.perf_counter() - t
        second = {'value': c2['jaccard_evals'] / dt2, 'cores': t2, 'seconds': dt2,
                  'sample': 'the same, at the box\'s CPU share per GPU'}
    return {'value': allc['jaccard_evals'] / dta, 'unit': 'Jaccard-evaluated read pairs/s', 'cores': threads,
            'kind': 'port', 'seconds': dta,
            'sample': f'oracle/fslr_oracle.c oracle_count_threads, all {csr.n_reads} query reads of the same input, '
                      f'{threads} threads sharing one index (index build included); {allc["jaccard_evals"]} '
                      f'Jaccard-evaluated pairs (GPU: {gpu_jacc})',
            'host_cpus_visible': os.cpu_count(),
            'cores_policy': cpu_policy(),
            'share_threads': second,
            'single_thread': {'value': one['jaccard_evals'] / dt1, 'cores': 1, 'seconds': dt1,
                              'sample': f'query reads of every {stride}th 64-rank block '
                                        f'({one["jaccard_evals"]} pairs, index build included)'},
            'reference_python': REFERENCE_PY}


if __name__ == '__main__':
    main()
