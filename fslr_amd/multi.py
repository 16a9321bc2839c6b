"""Multi-GPU clustering for the product path: ``fslr --skip-alignment --gpus N`` and
``cluster.query_interval_trees(..., n_gpus=N)`` (SURVEY.md §8b "Plus --backend/--gpus", §8e).

One process per GPU, as bench.py runs it.  A ``RankPool`` keeps ranks 1..N-1 alive as child
processes (``python -m fslr_amd.multi``): they are started before the calling process touches the
GPU — the CLI starts them before it reads the ``.mappings.bed`` file, so their interpreter, torch
import and process-group rendezvous overlap the host stages — and serve every query of the process.
The calling process is rank 0 (or one more child when this process already created a library
context but has not initialised torch's GPU runtime, whose bundled HIP runtime would then find no
device, or already belongs to a default process group).  Per query, the prepared CSR travels as
``.npy`` files in the pool's private directory (``/dev/shm`` when present; memory-mapped by the
children) and every rank runs one step of the chromosome-split sweep (dist.SweepShard, DESIGN.md
§6): it indexes and sweeps the chromosomes it owns, RCCL all_to_all routes the match entries to the
rank that owns each pair's first read, that rank evaluates the pair, and the ranks' edge lists are
all-gathered for the components.  When the reference's edge cap binds (cluster.py:223-224) the
candidates' loops are replayed sharded by the components of their hit graph, each rank replaying
its components and the ranks exchanging the rows their loops re-orient or drop.

Rank 0 returns the labels and the union of the ranks' edges and forward degrees (the children hand
theirs back through the same directory): they are the single-GPU results exactly.  An exception on
any rank (ZeroDivisionError where the reference raises it, a library error) is re-raised by the
caller with its type.

Process group: ``nccl`` (RCCL over xGMI) when there are at least N visible GPUs, rank r on device
(first + r) mod count; otherwise ``gloo`` with ranks sharing devices (the rehearsal mode bench.py /
tools/rehearse_multi.sh use on a one-GPU box), the exchange staged through host memory.
"""
from __future__ import annotations

import atexit
import json
import os
import shutil
import socket
import subprocess
import sys
import tempfile
import threading
import time

import numpy as np

_CSR_FIELDS = ('read_off', 'read_qlen2', 'read_nal', 'iv_chrom', 'iv_start', 'iv_end', 'iv_aln', 'data_pos')


def sweep_applies(csr, iv_thr) -> bool:
    """The chromosome split runs the sweep engine over each rank's chromosome filter: every folded
    overlap threshold >= 1 (overlap > 0), no aln_size == 0 interval and the intervals
    in the start-sorted data order the filter compacts (fslr_set_chrom_filter; any number of
    chromosomes).  Otherwise the ranks split the queries instead (dist.PairShard)."""
    t = np.asarray(iv_thr)
    return bool((t.size == 0 or t.min() >= 1) and getattr(csr, 'start_sorted', True))


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _save(d, csr, iv_thr, params):
    os.makedirs(d, exist_ok=True)
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


class _Rank:
    """One rank's process-group membership, device and stream, kept for every query of its pool."""

    def __init__(self, rank, world, port, first_device, force_gloo, timeout_s):
        from datetime import timedelta
        import torch
        import torch.distributed as dist
        from . import _lib
        n_dev = torch.cuda.device_count()
        if n_dev < 1:
            raise _lib.HipUnavailable('no HIP device visible')
        if dist.is_initialized():
            raise RuntimeError('a RankPool rank cannot join from a process that has a default process group')
        self.rank, self.world = rank, world
        self.backend = 'nccl' if n_dev >= world and not force_gloo else 'gloo'
        self.dev_index = (int(first_device) + rank) % n_dev
        self.dev = torch.device('cuda', self.dev_index)
        kw = dict(rank=rank, world_size=world, init_method=f'tcp://127.0.0.1:{port}',
                  timeout=timedelta(seconds=int(timeout_s)))
        if self.backend == 'nccl':
            kw['device_id'] = self.dev
        dist.init_process_group(self.backend, **kw)
        self.stream = torch.cuda.Stream(self.dev)
        self.ctx = None                               # the rank's library context, kept across queries

    def step(self, d):
        """One query on the CSR in directory d: the labels (every rank holds them), this rank's edges
        and forward degrees (capped ones when the cap bound).  The caller's current device and stream
        are restored."""
        import torch
        from . import _lib
        from .dist import PairShard, SweepShard, agree_error, chrom_counts_of
        from .prep import FSLR_MAX_L, FSLR_THR_ZERO_ALN, umax_table
        prev_dev = torch.cuda.current_device()
        prev_stream = torch.cuda.current_stream()
        torch.cuda.set_device(self.dev_index)
        torch.cuda.set_stream(self.stream)
        try:
            # per-query setup, then one agreement collective: a rank that fails here (context, upload,
            # chromosome filter) raises on every rank instead of leaving the others in the first
            # collective of the step until the group's timeout
            err = None
            try:
                csr, thr, pt, meta = _load(d)
                if self.ctx is None:
                    self.ctx = _lib.Context(self.dev_index, stream=self.stream.cuda_stream)
                rlen = np.diff(np.asarray(csr.read_off, np.int64))
                long_reads = bool(rlen.size and rlen.max() > FSLR_MAX_L)
                if sweep_applies(csr, thr) and not long_reads:
                    self.ctx.load_csr(csr, thr)
                    self.ctx.reserve_edges(max(1 << 16, 12 * csr.n_reads // self.world))
                    shard = SweepShard(self.ctx, csr.n_reads, chrom_counts_of(csr), self.world, self.rank, self.dev,
                                       split=meta.get('split', 'auto'))
                else:
                    # the query-shard split (dist.PairShard): every rank the full index
                    if long_reads:
                        self.ctx.load_csr_any(csr, np.where(np.asarray(csr.iv_aln) == 0, FSLR_THR_ZERO_ALN, 0))
                        self.ctx.set_thresholds(thr)
                        self.ctx.set_long_cutoffs(umax_table(meta['cutoffs'], int(rlen.max())))
                    else:
                        self.ctx.load_csr(csr, thr)
                    self.ctx.reserve_edges(max(1 << 16, 12 * csr.n_reads))
                    self.ctx.build_index()
                    shard = PairShard(self.ctx, csr.n_reads, self.world, self.rank, self.dev, long_reads=long_reads)
            except Exception as e:                   # noqa: BLE001 - raised on every rank by agree_error
                err = e
            try:
                agree_error(err, self.world, self.dev)
            except BaseException:
                if self.ctx is not None:
                    self.ctx.close()
                    self.ctx = None
                raise
            ctx = self.ctx
            try:
                info = shard.step(meta['qlen_cut'], meta['nal_cut'], pt, int(meta['edge_threshold']))
                torch.cuda.synchronize(self.dev)
                labels = shard.labels()
                if isinstance(shard, PairShard):
                    (a, b, I, U), fwd = shard.edges_out, shard.fwd_out
                else:
                    st = ctx.stats()
                    a, b, I, U = ctx.edges(st['n_edges'])
                    fwd = ctx.fwd_degree()
                return {'labels': labels, 'edges': (a, b, I, U), 'fwd': fwd, 'capped': bool(info['capped']),
                        'max_fwd': int(info['max_fwd']), 'cap': info.get('cap', {}), 'backend': self.backend,
                        'path': info['path'] if 'path' in info else 'sweep-' + shard.split}
            except BaseException:
                self.ctx.close()                      # a failed query leaves no half-set context behind
                self.ctx = None
                raise
        finally:
            torch.cuda.set_device(prev_dev)
            torch.cuda.set_stream(prev_stream)

    def close(self):
        import torch.distributed as dist
        if self.ctx is not None:
            self.ctx.close()
            self.ctx = None
        if dist.is_initialized():
            dist.destroy_process_group()


def _write_error(d, rank, e):
    with open(os.path.join(d, f'error{rank}.json'), 'w') as fh:
        json.dump({'type': type(e).__name__, 'msg': str(e)}, fh)


def _raise_error(d, rank):
    """Re-raise a rank's exception with its type (ZeroDivisionError as the reference raises it)."""
    from ._lib import FslrError, HipUnavailable
    path = os.path.join(d, f'error{rank}.json')
    if not os.path.exists(path):
        return
    with open(path) as fh:
        e = json.load(fh)
    kind = {'ZeroDivisionError': ZeroDivisionError, 'FslrError': FslrError, 'HipUnavailable': HipUnavailable,
            'ValueError': ValueError}.get(e['type'])
    if kind is not None:
        raise kind(e['msg'])
    raise RuntimeError(f'multi-GPU rank {rank}: {e["type"]}: {e["msg"]}')


def _child_loop(rank, world, port, first_device, force_gloo, timeout_s):
    """A pool rank: join the group once, then run each query named on stdin ('RUN dir'), answering
    'DONE' on stdout once its results (or its error) are in the directory; 'EXIT' ends it.  The
    protocol keeps the process's original stdout to itself: fd 1 is pointed at stderr, so what the
    libraries print (gloo's connection lines, warnings) cannot be read as an answer."""
    out = os.fdopen(os.dup(1), 'w', buffering=1)
    sys.stdout.flush()
    os.dup2(2, 1)
    r = None
    try:
        r = _Rank(rank, world, port, first_device, force_gloo, timeout_s)
        for line in sys.stdin:
            cmd = line.split()
            if not cmd or cmd[0] == 'EXIT':
                break
            d = cmd[1]
            try:
                res = r.step(d)
                a, b, I, U = res['edges']
                np.save(os.path.join(d, f'edges{rank}.npy'), np.stack([a, b, I, U]).astype(np.int32))
                np.save(os.path.join(d, f'fwd{rank}.npy'), res['fwd'])
                if rank == 0:                        # rank 0 run as a child: the caller's view too
                    np.save(os.path.join(d, 'labels0.npy'), np.asarray(res['labels'], np.int32))
                    with open(os.path.join(d, 'rank0.json'), 'w') as fh:
                        json.dump({k: res[k] for k in res if k not in ('edges', 'fwd', 'labels')}, fh, default=int)
            except Exception as e:                  # noqa: BLE001 - handed to the caller with its type
                _write_error(d, rank, e)
            out.write('DONE\n')
            out.flush()
    finally:
        if r is not None:
            r.close()
    return 0


def _rank0_in_process() -> bool:
    """Rank 0 runs in the calling process unless this library's HIP runtime is already up in it while
    torch's is not (torch bundles its own HIP runtime, which then finds no device; the reverse order
    works), or the caller already has a default process group (e.g. under torchrun)."""
    from . import _lib
    t = sys.modules.get('torch')
    if t is not None:
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            return False
    if not _lib.contexts_created():
        return True
    return bool(t is not None and t.cuda.is_initialized())


class RankPool:
    """Ranks 1..N-1 (and rank 0 when it cannot run in this process) as persistent child processes."""

    def __init__(self, world: int, first_device: int = 0, force_gloo: bool = False, timeout_s: int = 600):
        self.world = int(world)
        assert self.world >= 2
        self.first_device, self.force_gloo, self.timeout_s = int(first_device), bool(force_gloo), int(timeout_s)
        base = '/dev/shm' if os.path.isdir('/dev/shm') and os.access('/dev/shm', os.W_OK) else None
        self.dir = tempfile.mkdtemp(prefix='fslr_pool_', dir=base)
        self.port = _free_port()
        self.in_proc = _rank0_in_process()
        self.rank0 = None
        self.n_queries = 0
        env = dict(os.environ, MASTER_ADDR='127.0.0.1', MASTER_PORT=str(self.port))
        pkg_root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        env['PYTHONPATH'] = pkg_root + (os.pathsep + env['PYTHONPATH'] if env.get('PYTHONPATH') else '')
        self.procs = {}
        self._warm, self._warm_err = None, None
        for r in range(1 if self.in_proc else 0, self.world):
            self.procs[r] = subprocess.Popen(
                [sys.executable, '-m', 'fslr_amd.multi', str(r), str(self.world), str(self.port),
                 str(self.first_device), str(int(self.force_gloo)), str(self.timeout_s)],
                env=env, stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True, bufsize=1)
        if self.in_proc:
            # rank 0 joins on a worker thread (torch import, device, rendezvous) while the caller
            # reads and prepares its input; the first query waits for it
            self._warm = threading.Thread(target=self._make_rank0, daemon=True)
            self._warm.start()

    def _make_rank0(self):
        try:
            self.rank0 = _Rank(0, self.world, self.port, self.first_device, self.force_gloo, self.timeout_s)
        except BaseException as e:                   # noqa: BLE001 - raised by the first query
            self._warm_err = e

    def _wait_done(self, limit=None):
        """Every child's 'DONE' for the current query; RuntimeError when one died or, with ``limit``
        (seconds: rank 0 failed outside the collectives, so the others may wait for it forever),
        when they do not finish in time."""
        import select
        deadline = None if limit is None else time.monotonic() + limit
        pending = dict(self.procs)
        while pending:
            wait = None if deadline is None else max(0.0, deadline - time.monotonic())
            ready, _, _ = select.select([p.stdout for p in pending.values()], [], [], wait)
            if not ready:
                raise RuntimeError('multi-GPU ranks did not finish the query')
            for r, p in list(pending.items()):
                if p.stdout in ready:
                    line = p.stdout.readline().strip()
                    if line != 'DONE':
                        st = p.poll()
                        raise RuntimeError(f'multi-GPU rank {r} exited with status {st} during a query' if st is not None
                                           else f'multi-GPU rank {r} answered {line!r} instead of DONE')
                    del pending[r]

    def query(self, csr, iv_thr, qlen_cut, nal_cut, pass_table, edge_threshold, cutoffs=None, split='auto') -> dict:
        """One chromosome-split query; returns rank 0's view (labels, edges, fwd, capped, max_fwd, cap,
        backend)."""
        d = os.path.join(self.dir, f'q{self.n_queries}')
        self.n_queries += 1
        _save(d, csr, iv_thr, dict(qlen_cut=float(qlen_cut), nal_cut=float(nal_cut), pass_table=pass_table,
                                   edge_threshold=int(edge_threshold), split=split,
                                   cutoffs=None if cutoffs is None else [float(x) for x in cutoffs]))
        try:
            for p in self.procs.values():
                p.stdin.write(f'RUN {d}\n')
                p.stdin.flush()
            out = None
            err0 = None
            if self.in_proc:
                try:
                    if self._warm is not None:
                        self._warm.join()
                        self._warm = None
                        if self._warm_err is not None:
                            raise self._warm_err
                    if self.rank0 is None:
                        self.rank0 = _Rank(0, self.world, self.port, self.first_device, self.force_gloo,
                                           self.timeout_s)
                    out = self.rank0.step(d)
                except Exception as e:              # noqa: BLE001 - the children answer first
                    err0 = e
            if err0 is not None:
                try:
                    self._wait_done(limit=60)
                except RuntimeError:
                    self.close()
                raise err0
            self._wait_done()
            for r in self.procs:
                _raise_error(d, r)
            if out is None:
                with open(os.path.join(d, 'rank0.json')) as fh:
                    out = json.load(fh)
                out['labels'] = np.load(os.path.join(d, 'labels0.npy'))
                e = np.load(os.path.join(d, 'edges0.npy'))
                out['edges'] = tuple(e[k] for k in range(4))
                out['fwd'] = np.load(os.path.join(d, 'fwd0.npy'))
            parts = [out['edges']]
            fwd = np.asarray(out['fwd']).astype(np.int64)
            for r in range(1, self.world):
                e = np.load(os.path.join(d, f'edges{r}.npy'))
                parts.append(tuple(e[k] for k in range(4)))
                fwd += np.load(os.path.join(d, f'fwd{r}.npy'))
            out['edges'] = tuple(np.concatenate([p[k] for p in parts]).astype(np.int32) for k in range(4))
            out['fwd'] = fwd.astype(np.int32)
            return out
        except RuntimeError:
            self.close()                             # a rank that died leaves the group unusable
            raise
        finally:
            shutil.rmtree(d, ignore_errors=True)

    def alive(self) -> bool:
        return bool(self.procs) and all(p.poll() is None for p in self.procs.values())

    def close(self):
        for p in self.procs.values():
            try:
                if p.poll() is None:
                    p.stdin.write('EXIT\n')
                    p.stdin.flush()
            except (BrokenPipeError, OSError, ValueError):
                pass
        for p in self.procs.values():
            try:
                p.wait(timeout=10)                   # a rank still in the rendezvous never reads EXIT
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
        self.procs = {}
        if self._warm is not None and self._warm.is_alive():
            self._warm.join(timeout=5)               # its rendezvous fails once the other ranks are gone
        if self.rank0 is not None:
            self.rank0.close()
            self.rank0 = None
        shutil.rmtree(self.dir, ignore_errors=True)


_POOLS = {}


def pool(world: int, first_device: int = 0, force_gloo: bool = False) -> RankPool:
    """This process's pool of ``world`` ranks: started on first use (the CLI starts it before reading
    its input), restarted if a rank died."""
    key = (int(world), int(first_device), bool(force_gloo))
    p = _POOLS.get(key)
    if p is None or not p.alive():
        if p is not None:
            p.close()
        p = _POOLS[key] = RankPool(world, first_device, force_gloo)
    return p


@atexit.register
def close_pools():
    for p in list(_POOLS.values()):
        try:
            p.close()
        except Exception:                            # noqa: BLE001 - interpreter shutdown
            pass
    _POOLS.clear()


def query(csr, iv_thr, qlen_cut, nal_cut, pass_table, edge_threshold, n_gpus, first_device=0,
          force_gloo=False, cutoffs=None, split='auto') -> dict:
    """Run the chromosome-split query on ``n_gpus`` ranks of this process's pool; returns rank 0's view:
    ``labels`` (global min-rank labels), ``edges`` (a, b, I, U over all ranks), ``fwd`` (forward
    degrees), ``capped``, ``max_fwd``, ``backend``.  The pool's children start on the first call (or
    earlier, ``pool()``), before this process initialises the GPU."""
    global last_path
    rlen = np.diff(np.asarray(csr.read_off, np.int64))
    long_reads = bool(rlen.size and rlen.max() > 64)
    if split == 'auto':                       # SweepShard's resolution of 'auto'
        split = ('position' if int(n_gpus) > 1 and int(csr.n_chroms) <= 64 and getattr(csr, 'start_sorted', True)
                 else 'chrom')
    last_path = 'sweep-' + split if sweep_applies(csr, iv_thr) and not long_reads else ('long' if long_reads else 'walk')
    res = pool(n_gpus, first_device, force_gloo).query(csr, iv_thr, qlen_cut, nal_cut, pass_table, edge_threshold,
                                                       cutoffs=cutoffs, split=split)
    last_path = res.get('path') or last_path
    return res


last_path = None           # the split the last multi-GPU query took (tests: no one-GPU fallback)


if __name__ == '__main__':
    a = sys.argv[1:]
    sys.exit(_child_loop(int(a[0]), int(a[1]), int(a[2]), int(a[3]), bool(int(a[4])), int(a[5])))
