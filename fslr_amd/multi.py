"""Multi-GPU clustering for the product path: ``fslr --skip-alignment --gpus N`` and
``cluster.query_interval_trees(..., n_gpus=N)`` (SURVEY.md §8b "Plus --backend/--gpus", §8e).

One process per GPU, as bench.py runs it: the calling process is rank 0 and starts ranks
1..N-1 as child processes (``python -m fslr_amd.multi``) *before* it touches the GPU itself.
The prepared CSR travels through a private temporary directory of ``.npy`` files (memory-mapped
by the children).  Every rank runs one step of the chromosome-split sweep (dist.SweepShard,
DESIGN.md §6): it indexes and sweeps the chromosomes it owns, RCCL all_to_all routes the match
entries to the rank that owns each pair's first read, that rank evaluates the pair, and an RCCL
all_gather of the min-rank label vectors leaves the global components on every rank.  When the
reference's edge cap binds (cluster.py:223-224) rank 0 replays it on the whole input.

Rank 0 returns the labels and the union of the ranks' edges and forward degrees (the children
hand theirs back through the same directory); they are the single-GPU results exactly.

Process group: ``nccl`` (RCCL over xGMI) when there are at least N visible GPUs, rank r on
device (first + r) mod count; otherwise ``gloo`` with ranks sharing devices (the rehearsal mode
bench.py / tools/rehearse_multi.sh use on a one-GPU box), the exchange staged through host memory.
"""
from __future__ import annotations

import json
import os
import shutil
import socket
import subprocess
import sys
import tempfile
import time

import numpy as np

_CSR_FIELDS = ('read_off', 'read_qlen2', 'read_nal', 'iv_chrom', 'iv_start', 'iv_end', 'iv_aln', 'data_pos')


def sweep_applies(csr, iv_thr) -> bool:
    """The chromosome split runs the sweep engine over each rank's chromosome filter: every folded
    overlap threshold >= 1 (overlap > 0), no aln_size == 0 interval and the intervals
    in the start-sorted data order the filter compacts (fslr_set_chrom_filter; any number of
    chromosomes).  Otherwise the query runs on one GPU."""
    t = np.asarray(iv_thr)
    return bool((t.size == 0 or t.min() >= 1) and getattr(csr, 'start_sorted', True))


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _save(d, csr, iv_thr, params):
    for f in _CSR_FIELDS:
        np.save(os.path.join(d, f + '.npy'), np.asarray(getattr(csr, f)))
    np.save(os.path.join(d, 'iv_thr.npy'), np.asarray(iv_thr, dtype=np.int32))
    np.save(os.path.join(d, 'pass_table.npy'), np.asarray(params.pop('pass_table'), dtype=np.uint8))
    meta = dict(params, n_chroms=int(csr.n_chroms), start_sorted=bool(getattr(csr, 'start_sorted', True)))
    with open(os.path.join(d, 'params.json'), 'w') as fh:
        json.dump(meta, fh)


def _load(d):
    from .prep import CSR
    with open(os.path.join(d, 'params.json')) as fh:
        meta = json.load(fh)
    arr = {f: np.load(os.path.join(d, f + '.npy'), mmap_mode='r') for f in _CSR_FIELDS}
    n = arr['read_off'].shape[0] - 1
    csr = CSR(read_off=arr['read_off'], read_qlen2=arr['read_qlen2'], read_nal=arr['read_nal'],
              iv_chrom=arr['iv_chrom'], iv_start=arr['iv_start'], iv_end=arr['iv_end'], iv_aln=arr['iv_aln'],
              n_chroms=meta['n_chroms'], read_qcode=np.zeros(n, np.int64), data_pos=arr['data_pos'],
              nal_varies=False, start_sorted=meta['start_sorted'])
    thr = np.load(os.path.join(d, 'iv_thr.npy'))
    pt = np.load(os.path.join(d, 'pass_table.npy'))
    return csr, thr, pt, meta


def _rank_main(d: str, rank: int, world: int, port: int) -> dict:
    """One rank: join the process group, upload the CSR, run one SweepShard step."""
    from datetime import timedelta
    import torch
    import torch.distributed as dist
    from . import _lib
    from .dist import SweepShard, chrom_counts_of

    csr, thr, pt, meta = _load(d)
    n_dev = torch.cuda.device_count()
    if n_dev < 1:
        raise _lib.HipUnavailable('no HIP device visible')
    backend = 'nccl' if n_dev >= world and not meta.get('force_gloo') else 'gloo'
    dev_index = (int(meta.get('first_device', 0)) + rank) % n_dev
    torch.cuda.set_device(dev_index)
    dev = torch.device('cuda', dev_index)
    kw = dict(rank=rank, world_size=world, init_method=f'tcp://127.0.0.1:{port}',
              timeout=timedelta(seconds=int(meta.get('timeout_s', 300))))
    if backend == 'nccl':
        kw['device_id'] = dev
    dist.init_process_group(backend, **kw)
    try:
        stream = torch.cuda.Stream(dev)
        torch.cuda.set_stream(stream)
        ctx = _lib.Context(dev_index, stream=stream.cuda_stream)
        ctx.load_csr(csr, thr)
        ctx.reserve_edges(max(1 << 16, 12 * csr.n_reads // world))
        shard = SweepShard(ctx, csr.n_reads, chrom_counts_of(csr), world, rank, dev)
        info = shard.step(meta['qlen_cut'], meta['nal_cut'], pt, int(meta['edge_threshold']))
        torch.cuda.synchronize()
        labels = shard.labels()
        if info['capped'] and rank != 0:
            # rank 0 replayed the cap on the whole input: its context holds the whole graph
            a = b = I = U = np.zeros(0, np.int32)
            fwd = np.zeros(csr.n_reads, np.int32)
        else:
            st = ctx.stats()
            a, b, I, U = ctx.edges(st['n_edges'])
            fwd = ctx.fwd_degree()
        out = {'labels': labels, 'edges': (a, b, I, U), 'fwd': fwd, 'capped': bool(info['capped']),
               'max_fwd': int(info['max_fwd']), 'cap': info.get('cap', {}), 'backend': backend}
        dist.barrier()
        ctx.close()
        return out
    finally:
        dist.destroy_process_group()


def _child(d: str, rank: int, world: int, port: int) -> int:
    out = _rank_main(d, rank, world, port)
    a, b, I, U = out['edges']
    np.save(os.path.join(d, f'edges{rank}.npy'), np.stack([a, b, I, U]).astype(np.int32))
    np.save(os.path.join(d, f'fwd{rank}.npy'), out['fwd'])
    if rank == 0:                                  # rank 0 run as a child: the caller's view too
        np.save(os.path.join(d, 'labels0.npy'), np.asarray(out['labels'], np.int32))
        with open(os.path.join(d, 'rank0.json'), 'w') as fh:
            json.dump({k: out[k] for k in out if k not in ('edges', 'fwd', 'labels')}, fh, default=int)
    return 0


def _rank0_in_process() -> bool:
    """Rank 0 runs in the calling process unless this library's HIP runtime is already up in it while
    torch's is not: torch bundles its own HIP runtime, which then finds no device (the reverse order
    works), so rank 0 becomes a child process like the others."""
    from . import _lib
    if not _lib.contexts_created():
        return True
    t = sys.modules.get('torch')
    return bool(t is not None and t.cuda.is_initialized())


def query(csr, iv_thr, qlen_cut, nal_cut, pass_table, edge_threshold, n_gpus, first_device=0,
          timeout_s=300, force_gloo=False) -> dict:
    """Run the chromosome-split query on ``n_gpus`` ranks; returns rank 0's view: ``labels`` (global
    min-rank labels), ``edges`` (a, b, I, U over all ranks), ``fwd`` (forward degrees), ``capped``,
    ``max_fwd``, ``backend``.  Must be called before this process initialises the GPU (the children
    are started first)."""
    world = int(n_gpus)
    assert world >= 2
    d = tempfile.mkdtemp(prefix='fslr_multi_')
    procs = []
    try:
        _save(d, csr, iv_thr, dict(qlen_cut=float(qlen_cut), nal_cut=float(nal_cut), pass_table=pass_table,
                                   edge_threshold=int(edge_threshold), first_device=int(first_device),
                                   timeout_s=int(timeout_s), force_gloo=bool(force_gloo)))
        port = _free_port()
        env = dict(os.environ, MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
        pkg_root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        env['PYTHONPATH'] = pkg_root + (os.pathsep + env['PYTHONPATH'] if env.get('PYTHONPATH') else '')
        in_proc = _rank0_in_process()
        for r in range(0 if not in_proc else 1, world):
            procs.append(subprocess.Popen([sys.executable, '-m', 'fslr_amd.multi', d, str(r), str(world), str(port)],
                                          env=env))
        out = _rank_main(d, 0, world, port) if in_proc else None
        deadline = time.monotonic() + timeout_s
        for k, p in enumerate(procs):
            r = k + (1 if in_proc else 0)
            rc = p.wait(timeout=max(1.0, deadline - time.monotonic()))
            if rc != 0:
                raise RuntimeError(f'multi-GPU rank {r} exited with status {rc}')
        if out is None:
            with open(os.path.join(d, 'rank0.json')) as fh:
                out = json.load(fh)
            out['labels'] = np.load(os.path.join(d, 'labels0.npy'))
            e = np.load(os.path.join(d, 'edges0.npy'))
            out['edges'] = tuple(e[k] for k in range(4))
            out['fwd'] = np.load(os.path.join(d, 'fwd0.npy'))
        parts = [out['edges']]
        fwd = out['fwd'].astype(np.int64)
        for r in range(1, world):
            e = np.load(os.path.join(d, f'edges{r}.npy'))
            parts.append(tuple(e[k] for k in range(4)))
            fwd += np.load(os.path.join(d, f'fwd{r}.npy'))
        out['edges'] = tuple(np.concatenate([p[k] for p in parts]).astype(np.int32) for k in range(4))
        out['fwd'] = fwd.astype(np.int32)
        return out
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
        shutil.rmtree(d, ignore_errors=True)


if __name__ == '__main__':
    sys.exit(_child(sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])))
