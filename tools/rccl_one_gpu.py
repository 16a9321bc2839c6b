#!/usr/bin/env python3
"""RCCL through the product's multi-GPU step, two ranks sharing the one GPU of the box.

    python tools/rccl_one_gpu.py OUT.json [--reads 40000]

Each rank is a process with its own stream and library context on cuda:0, joined by
``torch.distributed`` with the nccl (RCCL) backend, and runs ``dist.SweepShard`` (split='auto') as
``bench.py --gpus 2`` does: two synchronous steps (entry counts exchanged, entries by
``all_to_all_single``, local forests by ``all_gather_into_tensor``, the agreement ``all_reduce``s —
every collective on device tensors through RCCL), then a repeat step and ``verify_repeat``.  Rank 0
checks the labels against one context's run of the whole input.  If RCCL refuses two ranks on one
device, the refusal is recorded instead (8-GPU runs are the driver's, SCALE_rNN.json).
"""
from __future__ import annotations

import datetime
import json
import os
import socket
import sys
import time
import traceback

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def _worker(rank, world, port, n_reads, out_dir):
    import torch
    import torch.distributed as dist
    res = {'rank': rank}
    try:
        os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
        dev = torch.device('cuda', 0)
        torch.cuda.set_device(dev)
        t0 = time.perf_counter()
        dist.init_process_group('nccl', rank=rank, world_size=world, device_id=dev,
                                timeout=datetime.timedelta(seconds=90))
        res['backend'] = dist.get_backend()
        x = torch.full((4,), rank + 1, dtype=torch.int64, device=dev)
        dist.all_reduce(x)
        torch.cuda.synchronize()
        res['all_reduce_ok'] = int(x[0].item()) == world * (world + 1) // 2
        res['init_s'] = time.perf_counter() - t0
        from fslr_amd import _lib, synth
        from fslr_amd.dist import SweepShard, chrom_counts_of
        from fslr_amd.prep import fold_overlap_threshold, pass_table
        s = synth.generate(n_reads, 16, 21)
        csr = s.interval_data().csr()
        stream = torch.cuda.Stream(dev)
        torch.cuda.set_stream(stream)
        ctx = _lib.Context(0, stream=stream.cuda_stream)
        thr = fold_overlap_threshold(csr.iv_aln, 0.8)
        ctx.load_csr(csr, thr)
        ctx.reserve_edges(max(1 << 16, 12 * csr.n_reads // world))
        sh = SweepShard(ctx, csr.n_reads, chrom_counts_of(csr), world, rank, dev, split='auto')
        pt = pass_table([1, 1, 0.66, 0.66, 0.66, 0.5])
        steps = []
        for _ in range(2):
            t = time.perf_counter()
            info = sh.step(1 - 0.04, 1 - 0.25, pt, 10)
            torch.cuda.synchronize()
            steps.append(time.perf_counter() - t)
        t = time.perf_counter()
        sh.step(1 - 0.04, 1 - 0.25, pt, 10, repeat=True)
        torch.cuda.synchronize()
        steps.append(time.perf_counter() - t)
        sh.verify_repeat()
        res.update(split=sh.split, step_s=steps, entries_sent=int(info['entries_sent']),
                   entries_received=int(info['entries_received']), capped=bool(info['capped']))
        labels = sh.labels()
        if rank == 0:
            ref = _lib.Context(0)
            ref.load_csr(csr, thr)
            ref.reserve_edges(12 * csr.n_reads)
            ref.run(1 - 0.04, 1 - 0.25, pt)
            res['labels_equal_single_context'] = bool(np.array_equal(labels, ref.labels()))
            res['n_reads'] = csr.n_reads
            ref.close()
        dist.barrier()
        ctx.close()
        dist.destroy_process_group()
        res['ok'] = True
    except Exception as e:                                   # noqa: BLE001 - recorded for the report
        res['ok'] = False
        res['error'] = f'{type(e).__name__}: {e}'
        res['trace'] = traceback.format_exc()[-2000:]
    with open(os.path.join(out_dir, f'rank{rank}.json'), 'w') as fh:
        json.dump(res, fh)


def main():
    import argparse
    import tempfile
    import torch.multiprocessing as mp
    ap = argparse.ArgumentParser()
    ap.add_argument('out')
    ap.add_argument('--reads', type=int, default=40_000)
    a = ap.parse_args()
    with socket.socket() as so:
        so.bind(('127.0.0.1', 0))
        port = so.getsockname()[1]
    with tempfile.TemporaryDirectory() as tmp:
        mp.spawn(_worker, args=(2, port, a.reads, tmp), nprocs=2, join=True)
        ranks = [json.load(open(os.path.join(tmp, f'rank{r}.json'))) for r in range(2)]
    out = {'what': 'dist.SweepShard over RCCL (nccl backend), 2 ranks sharing cuda:0', 'ranks': ranks}
    with open(a.out, 'w') as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps({r['rank']: {k: r.get(k) for k in ('ok', 'error', 'split', 'labels_equal_single_context',
                                                         'step_s')} for r in ranks}))


if __name__ == '__main__':
    main()
