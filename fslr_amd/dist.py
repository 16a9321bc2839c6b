"""Multi-GPU sharding (one process per GPU, torch.distributed over RCCL).

Two splits:

* SweepShard (the sweep engine, the default): every rank indexes and sweeps only the chromosomes it
  owns (chrom_owner: largest-first onto the least-loaded rank), and routes the match entries of
  each read pair to the rank owning the pair's first read (64-rank blocks dealt round robin) with
  one RCCL all_to_all; that rank evaluates the pair.  Exact because an interval only meets
  intervals of its own chromosome (cluster.py:159-160): a pair's first-fit matching is the union of
  its per-chromosome matchings, and all of them meet at one evaluator.  The index build, the sweep
  and the pair evaluation all split W ways.  Connectivity: the ranks' edge lists (8 B per edge)
  are all-gathered and every rank runs one union-find over their union (the replicated step).
* Query-read shards (the walk engine, fslr_query_shard): described next.

Query-read shards: query reads are split into blocks of SHARD_BLOCK
consecutive ranks dealt round robin to the processes (fslr_query_shard; low
ranks have more higher-rank partners, so contiguous ranges would not balance);
every process holds the full CSR and index in its HBM and evaluates the pairs
(A, B) with A in its shard and B > A.  Pair evaluation needs
no communication.  The one real exchange is connectivity: each process unions
its own edges into a forest whose labels are min-rank roots, the label vectors
(int32[N], 4 MB at 1M reads) are all-gathered over RCCL, and every process
unions (k, label_g[k]) for the other ranks g.  The union of per-shard
partitions is the partition of the union of edges, and min-rank roots do not
depend on the order of unions, so the result is identical to one GPU.

Forward degrees need no exchange for correctness (each read's forward edges are
all found by the shard that owns it); they are summed only for reporting.
"""
from __future__ import annotations

import os

import numpy as np


SHARD_BLOCK = 64     # query.hip kShardShift


def shard_of(reads, world: int):
    """Shard owning each read rank under fslr_query_shard (blocks of 64 ranks, round robin)."""
    return (np.asarray(reads) // SHARD_BLOCK) % world


def shard_range(n_reads: int, rank: int, world: int):
    """Contiguous, balanced [begin, end) of query read ranks for ``rank``."""
    base, rem = divmod(n_reads, world)
    begin = rank * base + min(rank, rem)
    return begin, begin + base + (1 if rank < rem else 0)


def union_find_labels(n: int, a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """Host union-find over edges: label = min element of the component (reference of the device forest)."""
    p = np.arange(n, dtype=np.int64)

    def find(x):
        r = x
        while p[r] != r:
            r = p[r]
        while p[x] != r:
            p[x], x = r, p[x]
        return r

    for x, y in zip(np.asarray(a).tolist(), np.asarray(b).tolist()):
        rx, ry = find(x), find(y)
        if rx != ry:
            if rx < ry:
                p[ry] = rx
            else:
                p[rx] = ry
    return np.array([find(i) for i in range(n)], dtype=np.int64)


def merge_label_sets(label_sets) -> np.ndarray:
    """Combine per-shard label vectors (each a partition of range(n)) into the finest
    common coarsening: union (k, labels_g[k]) for every shard g."""
    ls = [np.asarray(x, dtype=np.int64) for x in label_sets]
    n = ls[0].shape[0]
    src = np.concatenate([np.arange(n)] * len(ls))
    dst = np.concatenate(ls)
    return union_find_labels(n, src, dst)


class DeviceShardMerge:
    """Device-side label exchange for one step: copy local labels into a torch buffer,
    all_gather over the default process group (RCCL), union the other shards' labels
    into this context's forest and finalise.  All on the context's (= torch's current) stream."""

    def __init__(self, ctx, n_reads: int, world: int, rank: int, device):
        import torch
        self.ctx = ctx
        self.n = n_reads
        self.world = world
        self.rank = rank
        self.local = torch.empty(n_reads, dtype=torch.int32, device=device)
        self.gathered = torch.empty(world * n_reads, dtype=torch.int32, device=device)

    def __call__(self):
        import torch.distributed as dist
        self.ctx.copy_labels_device(self.local.data_ptr())
        if dist.get_backend() == 'gloo':
            # CPU-transport rehearsal (several ranks on one GPU): stage the exchange through host memory
            out = self.gathered.new_empty(self.gathered.shape, device='cpu')
            dist.all_gather_into_tensor(out, self.local.cpu())
            self.gathered.copy_(out)
        else:
            dist.all_gather_into_tensor(self.gathered, self.local)
        # one launch over all W label vectors (src = k mod n; this rank's own vector unions each
        # read with its own root, a no-op)
        self.ctx.union_pairs(None, self.gathered.data_ptr(), self.world * self.n, on_device=True)
        self.ctx.finalize_labels()


def chrom_owner(chrom_counts, world: int) -> np.ndarray:
    """Owner rank of each chromosome: largest interval count first onto the least-loaded rank
    (ties to the lower rank), so every rank's index and sweep cover about 1/W of the intervals."""
    cnt = np.asarray(chrom_counts, dtype=np.int64)
    owner = np.zeros(cnt.size, dtype=np.int64)
    load = np.zeros(world, dtype=np.int64)
    for c in sorted(range(cnt.size), key=lambda k: (-cnt[k], k)):
        r = int(np.argmin(load))
        owner[c] = r
        load[r] += cnt[c]
    return owner


POSITION_COST = 4       # per sorted position, in pair tests: the sweep's per-position work beside its tests
ENTRY_COST = 16         # per match entry, in pair tests: its write, partition, exchange and evaluation


def position_plan(tile_tests, tile_reach, n_intervals: int, world: int, per_position: int = POSITION_COST,
                  tile_entries=None, per_entry: int = ENTRY_COST):
    """Contiguous ranges of the (chrom, start)-sorted positions, one per rank: cut at 64-position tile
    boundaries where the running cost (the tile's pair tests, the sweep's work, plus ``per_position``
    per position and, given the tiles' match entries (fslr_position_entries), ``per_entry`` per entry)
    reaches r / world of the total, whatever the chromosomes.  Returns (lo, hi, end) per rank: the rank
    sweeps the pairs whose lower position lies in [lo, hi) and indexes [lo, end), end covering the
    forward windows of its tiles (fslr_position_costs).  Deterministic: every rank makes the same plan
    from its own full index."""
    tests = np.asarray(tile_tests, np.int64)
    reach = np.asarray(tile_reach, np.int64)
    nt = tests.size
    ni = int(n_intervals)
    width = np.minimum(64, ni - 64 * np.arange(nt, dtype=np.int64))
    cost = tests + per_position * width
    if tile_entries is not None:
        cost = cost + per_entry * np.asarray(tile_entries, np.int64)
    cum = np.cumsum(cost)
    total = int(cum[-1]) if nt else 0
    cuts = [0]
    for r in range(1, world):
        cuts.append(max(cuts[-1], min(nt, int(np.searchsorted(cum, total * r / world, side='left')) + 1)))
    cuts.append(nt)
    out = []
    for r in range(world):
        t0, t1 = cuts[r], cuts[r + 1]
        lo, hi = min(ni, 64 * t0), min(ni, 64 * t1)
        end = max(hi, int(reach[t0:t1].max())) if t1 > t0 else hi
        out.append((lo, hi, min(ni, end)))
    return out


def chrom_counts_of(csr) -> np.ndarray:
    return np.bincount(np.asarray(csr.iv_chrom), minlength=int(csr.n_chroms))


class TorchComm:
    """The step's collectives over the default process group (RCCL; with ``gloo`` the device tensors
    are staged through host memory: the one-GPU rehearsal and the CPU tests)."""

    def __init__(self, device):
        import torch
        self.device = torch.device(device)

    @property
    def gloo(self):
        import torch.distributed as dist
        return dist.get_backend() == 'gloo'

    def small(self, values):
        """An int64 tensor of ``values`` where this backend's small collectives take it."""
        import torch
        return torch.as_tensor(np.asarray(values, dtype=np.int64), device='cpu' if self.gloo else self.device)

    def all_to_all(self, out, inp, out_splits=None, in_splits=None):
        import torch.distributed as dist
        if self.gloo and out.device.type != 'cpu':
            o = out.cpu()
            dist.all_to_all_single(o, inp.cpu(), out_splits, in_splits)
            out.copy_(o)
        else:
            dist.all_to_all_single(out, inp, out_splits, in_splits)

    def all_gather(self, out, inp):
        import torch.distributed as dist
        if self.gloo and out.device.type != 'cpu':
            o = out.new_empty(out.shape, device='cpu')
            dist.all_gather_into_tensor(o, inp.cpu())
            out.copy_(o)
        else:
            dist.all_gather_into_tensor(out, inp)

    def all_reduce(self, t, op='max'):
        import torch.distributed as dist
        rop = {'max': dist.ReduceOp.MAX, 'min': dist.ReduceOp.MIN, 'sum': dist.ReduceOp.SUM}[op]
        if self.gloo and t.device.type != 'cpu':
            o = t.cpu()
            dist.all_reduce(o, op=rop)
            t.copy_(o)
        else:
            dist.all_reduce(t, op=rop)


class LocalHub:
    """In-process collectives for W ranks run as threads of one process, each with its own library
    context (tests: the product's SweepShard at W = 8 on one GPU).  A collective publishes each rank's
    tensor after a device synchronize, and every rank copies what it needs before the next one."""

    def __init__(self, world: int, timeout: float = 900.0):
        import threading
        self.world = int(world)
        self.barrier = threading.Barrier(self.world, timeout=timeout)
        self.slots = [None] * self.world

    def comm(self, rank: int, device):
        return LocalComm(self, rank, device)


class LocalComm:
    gloo = False

    def __init__(self, hub, rank, device):
        import torch
        self.hub, self.rank, self.device = hub, int(rank), torch.device(device)

    def small(self, values):
        import torch
        return torch.as_tensor(np.asarray(values, dtype=np.int64), device=self.device)

    def _sync(self):
        import torch
        if self.device.type == 'cuda':
            torch.cuda.synchronize(self.device)

    def _publish(self, obj):
        self._sync()
        self.hub.slots[self.rank] = obj
        self.hub.barrier.wait()
        return list(self.hub.slots)

    def _done(self):
        self._sync()
        self.hub.barrier.wait()

    def all_to_all(self, out, inp, out_splits=None, in_splits=None):
        W = self.hub.world
        if in_splits is None:
            in_splits = [inp.numel() // W] * W
        got = self._publish((inp, list(in_splits)))
        o = 0
        for t, spl in got:
            off, cnt = sum(spl[:self.rank]), spl[self.rank]
            out[o:o + cnt].copy_(t[off:off + cnt])
            o += cnt
        self._done()

    def all_gather(self, out, inp):
        n = inp.numel()
        got = self._publish(inp)
        for w, t in enumerate(got):
            out[w * n:(w + 1) * n].copy_(t[:n])
        self._done()

    def all_reduce(self, t, op='max'):
        import torch
        got = self._publish(t.clone())
        st = torch.stack([g.to(t.device) for g in got])
        if op == 'sum':
            t.copy_(st.sum(dim=0).to(t.dtype))
        else:
            t.copy_(st.max(dim=0).values if op == 'max' else st.min(dim=0).values)
        self._done()


def agree_error(err, world: int, device, comm=None):
    """MAX over ranks of an error code (0 none, 1 ZeroDivisionError, 2 other), one all_reduce: every
    rank raises together (its own exception, or one naming the other rank's) instead of leaving the
    others waiting in the next collective."""
    code = 0 if err is None else (1 if isinstance(err, ZeroDivisionError) else 2)
    if world > 1:
        comm = comm if comm is not None else TorchComm(device)
        t = comm.small([code])
        comm.all_reduce(t, 'max')
        code = int(t.item())
    if err is not None:
        raise err
    if code:
        from ._lib import FslrError
        raise ZeroDivisionError('division by zero') if code == 1 else FslrError('error on another rank')


class SweepShard:
    """One rank of the chromosome-split sweep (fslr_set_chrom_filter / fslr_sweep_partition /
    fslr_sweep_evaluate, then the edge exchange).  ``ctx`` holds every read (set_reads); this
    rank's index covers the chromosomes ``owner == rank``.  Entries travel as int64 tensors on
    ``device``; with the gloo backend they are staged through host memory (CPU rehearsal).

    step() leaves this rank's edges / forward degrees (pairs whose first read it owns) in ``ctx``
    and the global min-rank labels in ``ctx`` (labels()).  When the reference's edge cap binds
    (some read has more than ``edge_threshold`` forward edges) the graph depends on the sequential
    order of the reference's loops: the loops are replayed sharded over the ranks by the components
    of the candidates' hit graph (``capped`` in the step's result; ``ctx`` then holds this rank's
    capped edges, re-oriented as the reference's match rows, and their formers' edge counts).
    """

    def __init__(self, ctx, n_reads: int, chrom_counts, world: int, rank: int, device, block_shift: int = 6,
                 owner=None, comm=None, split: str = 'chrom'):
        """``split``: 'chrom' — each rank indexes and sweeps whole chromosomes (largest first onto the
        least-loaded rank); 'position' — each rank sweeps a contiguous range of sorted positions cut where
        the work balances (position_plan: pair tests, positions and match entries; one chromosome may
        span ranks), planned from one full index build and one counting sweep on the first step;
        'auto' — the position split when it applies (more than one rank, at most 64 chromosomes, the
        data-order index build), else the chromosome split.  The edge cap's sharded replay lists its
        hits on whole chromosomes in both (chrom_owner)."""
        import torch
        if split not in ('chrom', 'position', 'auto'):
            raise ValueError(f'split must be chrom, position or auto, not {split!r}')
        self._auto = split == 'auto'
        if self._auto:
            split = 'position' if int(world) > 1 and len(np.asarray(chrom_counts)) <= 64 else 'chrom'
        self.split = split
        self.pos = None                         # (lo, hi, end) of this rank once planned
        self.n_intervals = int(np.asarray(chrom_counts, np.int64).sum())
        self.ctx = ctx
        self.comm = comm if comm is not None else TorchComm(device)
        self.n = int(n_reads)
        self.world = int(world)
        self.rank = int(rank)
        self.device = torch.device(device)
        self.block_shift = int(block_shift)
        self.owner = chrom_owner(chrom_counts, world) if owner is None else np.asarray(owner)
        self.owned = self.owner == rank
        self.send = torch.empty(1 << 16, dtype=torch.int64, device=self.device)
        self.recv = torch.empty(1 << 16, dtype=torch.int64, device=self.device)
        self.local = torch.empty(self.n, dtype=torch.int32, device=self.device)
        self.esend = torch.empty(1 << 12, dtype=torch.int64, device=self.device)    # (a, b) int32 pairs
        self.egath = torch.empty(1 << 12, dtype=torch.int64, device=self.device)
        self._labels = None
        self._rep = None                   # the last synchronous step's counts (repeat steps)
        if split == 'chrom':
            ctx.set_chrom_filter(self.owned if world > 1 else None)

    def _plan_positions(self, qlen_cut, nal_cut, pass_table, edge_threshold):
        """The position split's range of this rank (every rank makes the same plan from its full index):
        cost = pair tests + per-position work + per-entry work, the entries from one counting sweep."""
        ctx = self.ctx
        ctx.set_chrom_filter(None)
        ctx.build_index()
        if self._auto and not ctx.has_data_order():
            # no data-order index build (fslr_set_reads_sorted inputs): the chromosome split, on every rank alike
            self.split = 'chrom'
            ctx.set_chrom_filter(self.owned if self.world > 1 else None)
            return
        tests, reach = ctx.position_costs()
        ent = ctx.position_entries(qlen_cut, nal_cut, pass_table, edge_threshold)
        self.plan = position_plan(tests, reach, self.n_intervals, self.world, tile_entries=ent)
        self.pos = self.plan[self.rank]
        self._plan_thr_gen = getattr(ctx, 'thr_gen', 0)
        ctx.set_position_filter(*self.pos)

    # -- collectives (self.comm: RCCL, gloo staged through host memory, or in-process) --------------
    def _all_to_all(self, out, inp, out_splits, in_splits):
        self.comm.all_to_all(out, inp, out_splits, in_splits)

    def _all_gather(self, out, inp):
        self.comm.all_gather(out, inp)

    def _grow(self, t, need):
        import torch
        if t.numel() >= need:
            return t
        return torch.empty(int(need * 1.125) + 4096, dtype=torch.int64, device=self.device)

    # -- one step -----------------------------------------------------------------------------
    def _key(self, qlen_cut, nal_cut, pass_table, edge_threshold):
        return (float(qlen_cut), float(nal_cut), np.asarray(pass_table, dtype=np.uint8).tobytes(), int(edge_threshold),
                getattr(self.ctx, 'thr_gen', 0))

    def step(self, qlen_cut, nal_cut, pass_table, edge_threshold=10, collect=False, repeat=False) -> dict:
        """One step.  ``collect``: also read the sweep's counters after the partition (one more
        sync; bench.py does it outside the timed steps).  ``repeat``: when the last step ran
        synchronously on this input with these parameters (and the cap did not bind), repeat it
        without host syncs: the partition lands where it did (fslr_sweep_partition_repeat, checked
        on the device), and the exchanges reuse its counts; verify_repeat() checks afterwards."""
        import torch
        ctx, W = self.ctx, self.world
        self._labels = None
        rep = self._rep if repeat else None
        if rep is not None and rep['key'] == self._key(qlen_cut, nal_cut, pass_table, edge_threshold):
            return self._step_repeat(qlen_cut, nal_cut, pass_table, edge_threshold, rep)
        self._rep = None
        err = None
        try:
            # plan again when the thresholds changed since: the halo covers the old sweep windows only
            if self.split == 'position' and (self.pos is None or
                                             self._plan_thr_gen != getattr(ctx, 'thr_gen', 0)):
                self._plan_positions(qlen_cut, nal_cut, pass_table, edge_threshold)
            ctx.build_index()
            ok, counts = ctx.sweep_partition(qlen_cut, nal_cut, pass_table, W, self.block_shift, self.send,
                                             edge_threshold)
            if not ok:
                self.send = self._grow(self.send, int(counts.sum()))
                ok, counts = ctx.sweep_partition(qlen_cut, nal_cut, pass_table, W, self.block_shift, self.send,
                                                 edge_threshold)
                assert ok
            if ctx.stats(check=False).get('overflow_flags', 0) & 64:
                # the ZeroDivisionError pair list overflowed (and grew): the cap replay needs all of them
                ok, counts = ctx.sweep_partition(qlen_cut, nal_cut, pass_table, W, self.block_shift, self.send,
                                                 edge_threshold)
                assert ok
        except Exception as e:                          # noqa: BLE001 - re-raised on every rank below
            if W == 1:
                raise
            # a negative count tells every destination (the counts exchange is the next collective)
            err = e
            counts = np.full(W, -1 if isinstance(e, ZeroDivisionError) else -2, dtype=np.int64)
        sweep_stats = ctx.stats(check=False) if collect and err is None else None
        sent_total = int(counts.sum())
        if W > 1:
            cin = self.comm.small(counts)
            cout = torch.empty_like(cin)
            self.comm.all_to_all(cout, cin)
            recv_counts = cout.cpu().numpy()
            if err is not None or (recv_counts < 0).any():
                if err is None:
                    from ._lib import FslrError
                    err = (ZeroDivisionError('division by zero') if (recv_counts == -1).any()
                           else FslrError('error on another rank'))
                raise err
            n_recv = int(recv_counts.sum())
            self.recv = self._grow(self.recv, n_recv)
            self._all_to_all(self.recv[:n_recv], self.send[:sent_total], recv_counts.tolist(), counts.tolist())
            entries = self.recv
        else:
            n_recv = sent_total
            entries = self.send
        err = None
        st = {'max_fwd': 0, 'n_edges': 0}
        try:
            # a failure here (NOMEM growing a buffer, a HIP error) rides in the all_reduce below, so
            # every rank raises instead of the others waiting in the next collective
            ctx.sweep_evaluate(qlen_cut, nal_cut, pass_table, entries, n_recv, edge_threshold)
            st = ctx.stats(check=False)
            while st['n_edges'] > st['edge_capacity']:
                ctx.reserve_edges(int(st['n_edges'] * 1.25) + 4096)
                ctx.sweep_evaluate(qlen_cut, nal_cut, pass_table, entries, n_recv, edge_threshold)
                st = ctx.stats(check=False)
            if st.get('error', 1) or st.get('overflow_flags', 1):   # only then read the stats again
                ctx.stats()                             # raises on a device-side error (ZeroDivisionError)
        except Exception as e:                          # noqa: BLE001 - re-raised on every rank below
            if W == 1:
                raise
            err = e
        mf = int(st['max_fwd'])
        max_ne = int(st['n_edges'])
        # pairs whose evaluation raises ZeroDivisionError, listed by this rank's partition sweep: the
        # reference raises when every loop runs to its end (the cap does not bind anywhere); otherwise
        # only where a capped loop reaches one (fslr_cap_local, the replay)
        zd = int(st.get('zd_pairs', 0))
        max_fp = 0
        if W > 1 and err is None and mf <= edge_threshold:
            # this rank's forest: the merge exchanges its pairs (not built when this rank already knows
            # the cap binds: the capped graph's forest replaces it)
            try:
                max_fp = ctx.local_forest()
            except Exception as e:                  # noqa: BLE001 - re-raised on every rank below
                err = e
        if W > 1:
            # the error flag, the edge count and the forest's pair count ride with the forward-degree
            # maximum, so a pair that raises on one evaluator raises on every rank instead of leaving
            # the others in a collective, and every rank knows the padded sizes of the exchanges
            code = 0 if err is None else (1 if isinstance(err, ZeroDivisionError) else 2)
            t = self.comm.small([mf, code, max_ne, max_fp, zd])
            self.comm.all_reduce(t, 'max')
            mf, code, max_ne, max_fp, zd = (int(x) for x in t.tolist())
            if err is None and code:
                from ._lib import FslrError
                err = ZeroDivisionError('division by zero') if code == 1 else FslrError('error on another rank')
        if err is None and zd > 0 and mf <= edge_threshold:
            err = ZeroDivisionError('division by zero')
        if err is not None:
            raise err
        out = {'entries_sent': sent_total, 'entries_received': n_recv, 'n_edges_local': int(st['n_edges']),
               'max_fwd': mf, 'capped': False, 'sweep_stats': sweep_stats}
        if mf > edge_threshold:
            out['capped'] = True
            out['cap'] = self._capped_labels(edge_threshold, max_ne)
            return out
        if W == 1:
            ctx.components()
            return out
        self._rep = {'key': self._key(qlen_cut, nal_cut, pass_table, edge_threshold), 'counts': counts.copy(),
                     'recv_counts': recv_counts.copy(), 'max_fp': max_fp, 'n_edges_local': int(st['n_edges']),
                     'out': dict(out, sweep_stats=None)}
        self._merge(max_fp)
        return out

    def _merge(self, max_fp):
        """Components of the union of the ranks' edges from their local forests: each rank's (read,
        root) pairs of the reads that are not their own root (fslr_local_forest; a partition is the
        union of the partitions of its parts, and a forest has fewer pairs than the edges it unions:
        about 0.37 of them at 1M reads) are all-gathered, padded to the largest count, and every rank
        unions them (8 B per pair)."""
        ctx, W = self.ctx, self.world
        m = max(1, max_fp)
        self.esend = self._grow(self.esend, m)
        self.egath = self._grow(self.egath, W * m)
        ctx.forest_pairs_into(self.esend, m)
        self._all_gather(self.egath[:W * m], self.esend[:m])
        ctx.components_from_pairs(self.egath, W * m)

    def _step_repeat(self, qlen_cut, nal_cut, pass_table, edge_threshold, rep) -> dict:
        """The last synchronous step again on unchanged input: the same kernels and exchanges, with
        the counts the synchronous step read back (the device checks its partition totals against
        them), so no host sync and no count exchange inside the step."""
        ctx, W = self.ctx, self.world
        counts, recv_counts = rep['counts'], rep['recv_counts']
        sent_total, n_recv = int(counts.sum()), int(recv_counts.sum())
        ctx.build_index()
        ctx.sweep_partition_repeat(qlen_cut, nal_cut, pass_table, W, self.block_shift, self.send, edge_threshold)
        self._all_to_all(self.recv[:n_recv], self.send[:sent_total], recv_counts.tolist(), counts.tolist())
        ctx.sweep_evaluate(qlen_cut, nal_cut, pass_table, self.recv, n_recv, edge_threshold)
        ctx.local_forest(count=False)
        self._merge(rep['max_fp'])
        self._rep_steps = getattr(self, '_rep_steps', 0) + 1
        return dict(rep['out'], repeat=True)

    def verify_repeat(self):
        """After repeat steps: every rank's device flags are clean (the partition totals equal the
        synchronous step's, no error) and its edge count is unchanged; raises on every rank otherwise."""
        rep = self._rep
        ok = 1
        err = None
        try:
            st = self.ctx.stats()                       # raises on a flagged repeat or a device error
            if rep is None or int(st['n_edges']) != rep['n_edges_local']:
                ok = 0
        except Exception as e:                          # noqa: BLE001 - re-raised below
            err = e
            ok = 0
        if self.world > 1:
            t = self.comm.small([ok])
            self.comm.all_reduce(t, 'min')
            ok = int(t.item())
        if err is not None:
            raise err
        if not ok:
            from ._lib import FslrError
            raise FslrError('a repeat step differed from the synchronous step on some rank')
        return True

    def _grow32(self, t, need):
        import torch
        if t is not None and t.numel() >= need:
            return t
        return torch.empty(int(need * 1.125) + 4096, dtype=torch.int32, device=self.device)

    def _agree(self, err):
        agree_error(err, self.world, self.device, self.comm)

    def _capped_labels(self, edge_threshold, max_ne):
        """The cap binds: the reference's graph depends on the sequential order of its loops
        (cluster.py:197-224).  Two loops depend on each other only when an interval of one read hits an
        interval of the other, so the loops are replayed sharded by the components of that graph over
        the candidates T (fslr_hip.h fslr_cap_install_pairs ... fslr_cap_apply_changes):

        1. every rank sorts its edges by lower read and gathers E* as (a, b) rows, computes the closure
           T over the rows' runs and lists the search-ordered hits of T's intervals on its own
           chromosomes;
        2. the ranks' local forests of the T-T hits (and T's hit counts) are all-gathered; every rank
           unions them and assigns the same components to ranks by cost;
        3. the lists travel to the rank replaying their read's component (all_to_all);
        4. each rank replays its components' loops and lists the rows they do not form in the lower
           read's loop (re-oriented or dropped);
        5. those changes are all-gathered and applied everywhere: each rank keeps its own capped edges
           and forward degrees (the reference's match rows); the ranks' local forests of those edges
           are merged as in the uncapped step, so every rank has the capped graph's labels.
        """
        import torch
        ctx, W, r = self.ctx, self.world, self.rank
        m = max(1, int(max_ne))
        err = None
        restricted = os.environ.get('FSLR_CAP_GATHER', 'restricted') != 'full'
        try:
            if not restricted:
                # every E* row travels: only this branch sizes the buffers for W * max_ne rows
                self.esend = self._grow(self.esend, m)
                self.egath = self._grow(self.egath, W * m)
                ctx.sort_edges()                 # each read's forward rows one run of the gathered rows
            else:
                # only the rows of S = {x : fwd(x) + bwd(x) >= threshold} travel (bwd summed over ranks)
                dt = (torch.uint8 if W * edge_threshold <= 255 and os.environ.get('FSLR_CAP_BWD') != 'i32'
                      else torch.int32)
                if getattr(self, 'bwd', None) is None or self.bwd.dtype != dt or self.bwd.numel() < self.n:
                    self.bwd = torch.empty(max(1, self.n), dtype=dt, device=self.device)
                ctx.cap_bwd_counts(edge_threshold, self.bwd)
        except Exception as e:                   # noqa: BLE001 - re-raised on every rank
            err = e
        self._agree(err)
        if restricted:
            if W > 1:
                self.comm.all_reduce(self.bwd[:self.n], 'sum')
            nr = 0
            try:
                nr = ctx.cap_restrict(self.bwd)
            except Exception as e:               # noqa: BLE001
                err = e
            code = 0 if err is None else (1 if isinstance(err, ZeroDivisionError) else 2)
            if W > 1:
                t = self.comm.small([code, nr])
                self.comm.all_reduce(t, 'max')
                code, m = (int(x) for x in t.tolist())
            else:
                m = nr
            if err is not None:
                raise err
            if code:
                from ._lib import FslrError
                raise FslrError('error on another rank')
            m = max(1, m)
            self.esend = self._grow(self.esend, m)
            self.egath = self._grow(self.egath, W * m)
            ctx.cap_copy_restricted(self.esend, m)
        else:
            ctx.edges_into(self.esend, m)
        if W > 1:
            self._all_gather(self.egath[:W * m], self.esend[:m])
            rows = self.egath
        else:
            rows = self.esend
        nt = 0
        try:
            if restricted:
                ctx.cap_install_restricted(rows, W * m, W, r)
            else:
                ctx.cap_install_pairs(rows, W * m, W, r)
            if self.split == 'position':
                # the replay lists each interval's hits in search order from one index holding its whole
                # chromosome: the chromosome split's index for this step (the next step's build restores
                # the position range)
                ctx.set_chrom_filter(self.owned if W > 1 else None)
                ctx.build_index()
            ctx.cap_local(edge_threshold)
            nt = ctx.cap_sizes()[0]
            self.tinfo = self._grow32(getattr(self, 'tinfo', None), max(1, 2 * nt))
            ctx.cap_dep_local(self.tinfo)
        except Exception as e:                          # noqa: BLE001 - re-raised on every rank
            err = e
        self._agree(err)
        if W > 1:
            self.tgath = self._grow32(getattr(self, 'tgath', None), max(1, W * 2 * nt))
            if nt:
                self._all_gather(self.tgath[:W * 2 * nt], self.tinfo[:2 * nt])
            tg = self.tgath
        else:
            tg = self.tinfo
        ti_d = hits_d = np.zeros(W, np.int64)
        try:
            ti_d, hits_d = ctx.cap_shard_plan(tg, W, r)
            self.csend = self._grow32(getattr(self, 'csend', None), max(1, int(ti_d.sum())))
            self.hsend = self._grow32(getattr(self, 'hsend', None), max(1, int(hits_d.sum())))
            ctx.cap_shard_pack(self.csend, self.hsend)
        except Exception as e:                          # noqa: BLE001
            err = e
        self._agree(err)
        nmine = int(ti_d[r])
        if W > 1:
            self.crecv = self._grow32(getattr(self, 'crecv', None), max(1, W * nmine))
            self._all_to_all(self.crecv[:W * nmine], self.csend[:int(ti_d.sum())], [nmine] * W, ti_d.tolist())
            hin = self.comm.small(hits_d)
            hout = torch.empty_like(hin)
            self._all_to_all(hout, hin, [1] * W, [1] * W)
            hits_from = hout.cpu().numpy()
            self.hrecv = self._grow32(getattr(self, 'hrecv', None), max(1, int(hits_from.sum())))
            self._all_to_all(self.hrecv[:int(hits_from.sum())], self.hsend[:int(hits_d.sum())], hits_from.tolist(),
                             hits_d.tolist())
            rcnt, rhits = self.crecv, self.hrecv
        else:
            rcnt, rhits = self.csend, self.hsend
        nch, part = 0, {}
        try:
            nch, part = ctx.cap_replay_shard(rcnt, rhits)
        except Exception as e:                          # noqa: BLE001
            err = e
        # the error code rides with the change count and the partial statistics
        code = 0 if err is None else (1 if isinstance(err, ZeroDivisionError) else 2)
        mine = np.array([code, nch, part.get('capped', 0), part.get('hits', 0), part.get('pairs', 0)], np.int64)
        if W > 1:
            t = self.comm.small(mine)
            g = torch.empty(5 * W, dtype=torch.int64, device=t.device)
            self._all_gather(g, t)
            allp = g.cpu().numpy().reshape(W, 5)
        else:
            allp = mine.reshape(1, 5)
        if err is not None:
            raise err
        if allp[:, 0].max():
            from ._lib import FslrError
            raise ZeroDivisionError('division by zero') if (allp[:, 0] == 1).any() else FslrError('error on another rank')
        pad = max(1, int(allp[:, 1].max()))
        self.chsend = self._grow32(getattr(self, 'chsend', None), pad)
        ctx.cap_copy_changes(self.chsend, pad)
        if W > 1:
            self.chgath = self._grow32(getattr(self, 'chgath', None), W * pad)
            self._all_gather(self.chgath[:W * pad], self.chsend[:pad])
            chg = self.chgath
        else:
            chg = self.chsend
        cap = {}
        fp = 0
        try:
            cap = ctx.cap_apply_changes(chg, W * pad)
            cap.update(capped=int(allp[:, 2].sum()), hits=int(allp[:, 3].sum()), pairs=int(allp[:, 4].sum()))
            if W == 1:
                ctx.components()
            else:
                fp = ctx.local_forest()             # the capped graph's components: the forest merge
        except Exception as e:                          # noqa: BLE001
            err = e
        if W > 1:
            code = 0 if err is None else (1 if isinstance(err, ZeroDivisionError) else 2)
            # the restricted gather's max_fwd is this rank's part (S and its own reads outside S)
            t = self.comm.small([code, fp, int(cap.get('max_fwd', 0))])
            self.comm.all_reduce(t, 'max')
            code, fp, mf = (int(x) for x in t.tolist())
            if cap:
                cap['max_fwd'] = mf
            if err is None and code:
                from ._lib import FslrError
                err = ZeroDivisionError('division by zero') if code == 1 else FslrError('error on another rank')
            if err is None:
                self._merge(fp)
        if self.split == 'position':
            ctx.use_position_filter()
        if err is not None:
            raise err
        return cap

    def labels(self) -> np.ndarray:
        """Global min-rank labels after step() (every rank)."""
        return self._labels if self._labels is not None else self.ctx.labels()


class PairShard(SweepShard):
    """One rank of the query-shard split for the inputs the sweep split does not take:
    overlap <= 0 (matches need not overlap), an aln_size == 0 interval, reads of more than FSLR_MAX_L
    intervals.  Every rank holds every read and the full index and decides the pairs whose lower-rank
    read lies in its blocks of 64 ranks (dealt round robin) — the walk engine's fslr_query_shard, or with
    long reads the general evaluator's fslr_long_pairs_shard — so each pair is decided once
    (cluster.py:197-208: a pair is first met from its lower-rank read's loop when no loop breaks).
    Components merge by the ranks' local forests (as SweepShard).  ZeroDivisionError pairs are listed
    per rank and raise on every rank when the cap does not bind anywhere.  When it binds, E* is gathered
    and every rank replays the reference's loops over it (fslr_apply_edge_cap /
    fslr_cap_replay_pairs); each rank then reports the capped edges and forward degrees of its own
    read blocks, so the ranks' parts still add up to the one-GPU graph."""

    def __init__(self, ctx, n_reads: int, world: int, rank: int, device, comm=None, long_reads: bool = False):
        import torch
        self.ctx = ctx
        self.comm = comm if comm is not None else TorchComm(device)
        self.n = int(n_reads)                   # real reads
        self.world, self.rank = int(world), int(rank)
        self.device = torch.device(device)
        self.long = bool(long_reads)
        self.split = 'query'
        self.esend = torch.empty(1 << 12, dtype=torch.int64, device=self.device)
        self.egath = torch.empty(1 << 12, dtype=torch.int64, device=self.device)
        self._labels = None
        self._rep = None
        self.edges_out = None                   # (a, b, I, U) of this rank's part (host)
        self.fwd_out = None

    def _mine(self, reads):
        return (np.asarray(reads, np.int64) >> 6) % self.world == self.rank

    def step(self, qlen_cut, nal_cut, pass_table, edge_threshold=10, **_) -> dict:
        import torch
        ctx, W, r = self.ctx, self.world, self.rank
        thr = int(edge_threshold)
        self._labels = None
        err = None
        mf = zd = ne = 0
        part = None
        try:
            if self.long:
                n_long = ctx.long_pairs_shard(qlen_cut, nal_cut, pass_table, r, W, thr)
                st = ctx.stats(check=False)
                if st.get('overflow_flags', 0) & 64:   # the ZeroDivisionError list grew: list them all
                    n_long = ctx.long_pairs_shard(qlen_cut, nal_cut, pass_table, r, W, thr)
                    st = ctx.stats(check=False)
                part = ctx.long_edges(n_long)
                ne = int(n_long)
                mf = int(np.bincount(part[0], minlength=1).max()) if ne else 0
            else:
                while True:
                    ctx.query_shard(qlen_cut, nal_cut, pass_table, r, W, thr)
                    st = ctx.stats(check=False)
                    grow = False
                    if st['n_edges'] > st['edge_capacity']:
                        ctx.reserve_edges(int(st['n_edges'] * 1.25) + 4096)
                        grow = True
                    if st['deferred'] > st['deferred_capacity']:
                        ctx.reserve_deferred(int(st['deferred'] * 1.25) + 4096)
                        grow = True
                    if st.get('overflow_flags', 0) & 64:  # the ZeroDivisionError list grew: list them all
                        grow = True
                    if not grow:
                        break
                ne = int(st['n_edges'])
                mf = int(st['max_fwd'])
            zd = int(st.get('zd_pairs', 0))
        except Exception as e:                         # noqa: BLE001 - re-raised on every rank below
            if W == 1:
                raise
            err = e
        code = 0 if err is None else (1 if isinstance(err, ZeroDivisionError) else 2)
        if W > 1:
            t = self.comm.small([mf, code, zd, ne])
            self.comm.all_reduce(t, 'max')
            mf, code, zd, ne_max = (int(x) for x in t.tolist())
        else:
            ne_max = ne
        if err is None and code:
            from ._lib import FslrError
            err = ZeroDivisionError('division by zero') if code == 1 else FslrError('error on another rank')
        if err is None and zd > 0 and mf <= thr:
            err = ZeroDivisionError('division by zero')   # every loop runs to its end: each pair is visited
        if err is not None:
            raise err
        out = {'capped': mf > thr, 'max_fwd': mf, 'n_edges_local': ne, 'path': 'long' if self.long else 'walk'}
        if mf <= thr:
            if self.long:
                a, b, I, U = part
                self.edges_out = (a, b, I, U)
            else:
                self.edges_out = ctx.edges(ne)
            fwd = np.bincount(self.edges_out[0], minlength=self.n)[:self.n]
            self.fwd_out = fwd.astype(np.int32)
            if W > 1:
                fp = ctx.local_forest()                # the merge unions the ranks' forests
                t = self.comm.small([fp])
                self.comm.all_reduce(t, 'max')
                self._merge(int(t.item()))
            else:
                ctx.components()
            self._labels = ctx.labels()[:self.n]
            return out
        cap, err = {}, None
        try:
            cap = self._capped(thr, part, ne_max)
        except Exception as e:                         # noqa: BLE001 - a replayed loop raised on some rank
            err = e
        self._agree(err)
        out['cap'] = cap
        return out

    def _capped(self, thr, part, ne_max):
        """The cap binds: E* on every rank, the loops replayed on each (the same result everywhere)."""
        import torch
        ctx, W = self.ctx, self.world
        m = max(1, int(ne_max))
        if self.long:
            a, b, I, U = part
            rows = np.full((m, 4), -1, np.int32)
            rows[:a.size] = np.stack([a, b, I, U], axis=1)
            t = torch.from_numpy(rows.reshape(-1).view(np.int64).copy()).to(self.device)
            g = torch.empty(W * t.numel(), dtype=torch.int64, device=self.device)
            if W > 1:
                self._all_gather(g, t)
            else:
                g = t
            allr = g.cpu().numpy().view(np.int32).reshape(-1, 4)
            allr = allr[allr[:, 0] >= 0]
            order = np.lexsort((allr[:, 1], allr[:, 0]))
            allr = allr[order]
            a, b, I, U = (allr[:, k].copy() for k in range(4))
            who, fwd, cap = ctx.cap_replay_pairs(thr, a, b, self.n)
            keep = who != 2
            a2, b2 = np.where(who == 0, a, b)[keep], np.where(who == 0, b, a)[keep]
            I2, U2 = I[keep], U[keep]
            ctx.components()
            self._labels = ctx.labels()[:self.n]
        else:
            self.esend = self._grow(self.esend, 2 * m)            # rows of 16 B: two int64 per row
            self.egath = self._grow(self.egath, 2 * W * m)
            ctx.edges_iu_into(self.esend, m)
            if W > 1:
                self._all_gather(self.egath[:2 * W * m], self.esend[:2 * m])
                rows = self.egath
            else:
                rows = self.esend
            ctx.cap_install_edges(rows, W * m)
            cap = ctx.apply_edge_cap(thr)
            st = ctx.stats()
            a2, b2, I2, U2 = ctx.edges(st['n_edges'])
            fwd = ctx.fwd_degree()
            ctx.components()
            self._labels = ctx.labels()[:self.n]
        mine = self._mine(a2)
        self.edges_out = (a2[mine], b2[mine], I2[mine], U2[mine])
        f = np.asarray(fwd, np.int64)[:self.n].copy()
        f[~self._mine(np.arange(self.n))] = 0
        self.fwd_out = f.astype(np.int32)
        return cap

    def labels(self) -> np.ndarray:
        return self._labels
