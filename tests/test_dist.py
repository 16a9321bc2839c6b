"""Multi-GPU path: query-read row shards + label exchange.

CPU tests run the real torch.distributed exchange over gloo with world_size 2 (two spawned
processes on 127.0.0.1); the shard-local edges come from the CPU oracle restricted to each
shard's query reads.  The GPU test drives fslr_amd.dist.DeviceShardMerge with two contexts on
one card (the all-gather is done in-process), so the device union / finalize path is exercised
exactly as bench.py uses it.
"""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest

from fslr_amd import synth
from fslr_amd.dist import merge_label_sets, shard_of, shard_range, union_find_labels
from oracle import oracle as O


def _oracle_csr(c):
    cnt = np.diff(c.read_off)
    return O.OracleCSR(c.read_off, c.iv_chrom, c.iv_start, c.iv_end, c.iv_aln, np.repeat(c.read_qlen2, cnt),
                       np.repeat(c.read_nal, cnt), c.data_pos)


def _components_from_labels(lab):
    """Oracle numbering (first insertion == min rank) from min-rank labels; -1 = singleton."""
    n = lab.shape[0]
    sizes = np.bincount(lab, minlength=n)
    roots = np.flatnonzero(sizes >= 2)
    rid = np.full(n, -1)
    rid[roots] = np.arange(roots.size)
    return np.where(sizes[lab] >= 2, rid[lab], -1)


def test_shard_range_partitions_ranks():
    for n in (0, 1, 7, 1000, 1_000_003):
        for world in (1, 2, 3, 8):
            rs = [shard_range(n, r, world) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            for (a0, a1), (b0, _) in zip(rs, rs[1:]):
                assert a1 == b0
            sizes = [b - a for a, b in rs]
            assert max(sizes) - min(sizes) <= 1


@pytest.fixture(scope='module')
def world_case():
    s = synth.generate(6000, 8, 31)
    csr = s.interval_data().csr()
    o = O.run_core(_oracle_csr(csr), use_cap=False)
    return csr, o


def test_shard_of_balances_and_partitions():
    n = 1_000_003
    for world in (2, 3, 8):
        sh = shard_of(np.arange(n), world)
        counts = np.bincount(sh, minlength=world)
        assert counts.sum() == n and counts.max() - counts.min() <= 64


def test_shards_partition_evaluated_pairs(world_case):
    """Pairs are owned by their lower-rank read: per-shard oracle counts add up to the whole."""
    csr, o = world_case
    oc = _oracle_csr(csr)
    n = csr.n_reads
    prev = 0
    total = 0
    for r in range(3):
        _, a1 = shard_range(n, r, 3)
        cum = O.run_core(oc, use_cap=False, query_end=a1)['stats']['evaluated_pairs']
        total += cum - prev
        prev = cum
    assert total == o['stats']['evaluated_pairs']


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _gloo_worker(rank, world, port, n, ea, eb, out_dir):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    mine = shard_of(ea, world) == rank
    local = union_find_labels(n, ea[mine], eb[mine])
    t = torch.from_numpy(local.astype(np.int64))
    gathered = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(gathered, t)
    merged = merge_label_sets([g.numpy() for g in gathered])
    np.save(os.path.join(out_dir, f'rank{rank}.npy'), merged)
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_merge_equals_single_process_components(world_case, tmp_path):
    import torch.multiprocessing as mp
    csr, o = world_case
    n = csr.n_reads
    ea, eb = o['edge_a'].astype(np.int64), o['edge_b'].astype(np.int64)
    assert ea.size > 100
    mp.start_processes(_gloo_worker, args=(2, _free_port(), n, ea, eb, str(tmp_path)), nprocs=2, join=True,
                       start_method='spawn')
    full = union_find_labels(n, ea, eb)
    for r in range(2):
        got = np.load(tmp_path / f'rank{r}.npy')
        np.testing.assert_array_equal(got, full)
        np.testing.assert_array_equal(_components_from_labels(got), o['comp'])


@pytest.mark.gpu
def test_device_shard_merge_two_contexts_one_gpu(monkeypatch):
    """Two shard contexts on cuda:0; DeviceShardMerge with an in-process all-gather must give
    every shard the single-context labels (and the oracle's components)."""
    import torch
    import torch.distributed as dist
    from fslr_amd import _lib
    from fslr_amd.dist import DeviceShardMerge
    from fslr_amd.prep import fold_overlap_threshold, pass_table

    s = synth.generate(30_000, 16, 8)
    csr = s.interval_data().csr()
    n = csr.n_reads
    thr = fold_overlap_threshold(csr.iv_aln, 0.8)
    pt = pass_table([1, 1, 0.66, 0.66, 0.66, 0.5])
    dev = torch.device('cuda', 0)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    ctxs, merges = [], []
    for r in range(2):
        c = _lib.Context(0, stream=stream.cuda_stream)
        c.load_csr(csr, thr)
        c.reserve_edges(12 * n)
        c.set_shard(r, 2)                # shard-restricted query-side index data, as bench.py
        c.build_index()
        c.query_shard(1 - 0.04, 1 - 0.25, pt, r, 2)
        c.components()
        ctxs.append(c)
        merges.append(DeviceShardMerge(c, n, 2, r, dev))
    # in-process all-gather: rank r's local labels land in slot r of every rank's buffer
    for m in merges:
        m.ctx.copy_labels_device(m.local.data_ptr())
    locals_ = [m.local.clone() for m in merges]

    def fake_all_gather(out, inp):
        out.copy_(torch.cat(locals_))

    monkeypatch.setattr(dist, 'all_gather_into_tensor', fake_all_gather)
    monkeypatch.setattr(dist, 'get_backend', lambda *a, **k: 'nccl')
    for m in merges:
        m()
    torch.cuda.synchronize()
    ref = _lib.Context(0)
    ref.load_csr(csr, thr)
    ref.reserve_edges(12 * n)
    ref.run(1 - 0.04, 1 - 0.25, pt)
    want = ref.labels()
    o = O.run_core(_oracle_csr(csr), use_cap=False)
    for c in ctxs:
        got = c.labels()
        np.testing.assert_array_equal(got, want)
        np.testing.assert_array_equal(_components_from_labels(got), o['comp'])
    st = [c.stats() for c in ctxs]
    assert sum(x['evaluated_pairs'] for x in st) == o['stats']['evaluated_pairs']
    assert sum(x['n_edges'] for x in st) == o['edge_a'].size
    # each shard's edges are exactly the oracle edges whose lower-rank read it owns
    for r, c in enumerate(ctxs):
        a, b, I, U = c.edges(st[r]['n_edges'])
        mine = shard_of(o['edge_a'], 2) == r
        assert sorted(zip(a.tolist(), b.tolist())) == sorted(zip(o['edge_a'][mine].tolist(), o['edge_b'][mine].tolist()))
    for c in ctxs + [ref]:
        c.close()


# ---- chromosome-split sweep (dist.SweepShard) ----------------------------------------------------

def test_chrom_owner_balances():
    from fslr_amd.dist import chrom_owner
    cnt = np.array([100] * 23)
    for world in (1, 2, 3, 8):
        own = chrom_owner(cnt, world)
        load = np.bincount(own, weights=cnt, minlength=world)
        assert load.max() - load.min() <= 100
    own = chrom_owner([5, 90, 10, 40, 50], 2)
    load = np.bincount(own, weights=[5, 90, 10, 40, 50], minlength=2)
    assert sorted(load.tolist()) == [95, 100]


def test_emulated_sweep_split_equals_oracle(world_case):
    """The decomposition itself, in one process: entries of each rank's chromosomes, routed by
    first-read block, evaluated per destination — the union of the destinations' edges is the
    oracle's edge set (with I, U), and no pair is evaluated twice."""
    import torch
    from fslr_amd.dist import chrom_counts_of, chrom_owner
    from fslr_amd.prep import fold_overlap_threshold, pass_table
    from tests.sweep_emu import EmuSweepContext
    csr, o = world_case
    thr = fold_overlap_threshold(csr.iv_aln, 0.8)
    pt = pass_table([1, 1, 0.66, 0.66, 0.66, 0.5])
    W = 3
    owner = chrom_owner(chrom_counts_of(csr), W)
    parts = [[] for _ in range(W)]
    for r in range(W):
        e = EmuSweepContext(csr, thr)
        e.set_chrom_filter(owner == r)
        buf = torch.empty(1 << 22, dtype=torch.int64)
        ok, counts = e.sweep_partition(1 - 0.04, 1 - 0.25, pt, W, 6, buf)
        assert ok
        pos = np.concatenate([[0], np.cumsum(counts)])
        for d in range(W):
            parts[d].append(buf[pos[d]:pos[d + 1]].clone())
    got = []
    for d in range(W):
        e = EmuSweepContext(csr, thr)
        ent = torch.cat(parts[d])
        assert ((ent >> (39 + 6)) % W == d).all()
        e.sweep_evaluate(1 - 0.04, 1 - 0.25, pt, ent, ent.numel())
        a, b, I, U = e.edges(e.stats()['n_edges'])
        got += list(zip(a.tolist(), b.tolist(), I.tolist(), U.tolist()))
    want = sorted(zip(o['edge_a'].tolist(), o['edge_b'].tolist(), o['edge_I'].tolist(), o['edge_U'].tolist()))
    assert len(got) == len(set(got))
    assert sorted(got) == want


def _sweep_worker(rank, world, port, csr, thr, out_dir, edge_threshold):
    import torch.distributed as dist
    from fslr_amd.dist import SweepShard, chrom_counts_of
    from fslr_amd.prep import pass_table
    from tests.sweep_emu import EmuSweepContext
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    ctx = EmuSweepContext(csr, thr)
    sh = SweepShard(ctx, csr.n_reads, chrom_counts_of(csr), world, rank, 'cpu')
    pt = pass_table([1, 1, 0.66, 0.66, 0.66, 0.5])
    info = sh.step(1 - 0.04, 1 - 0.25, pt, edge_threshold)
    # a repeat step (no host syncs: the synchronous step's counts) gives the same result; with the
    # cap binding it runs synchronously again
    info2 = sh.step(1 - 0.04, 1 - 0.25, pt, edge_threshold, repeat=True)
    assert info2.get('repeat', False) == (not info['capped'])
    if info2.get('repeat'):
        assert ctx.repeat_partitions == 1
        sh.verify_repeat()
    np.save(os.path.join(out_dir, f'labels{rank}.npy'), sh.labels())
    a, b, I, U = ctx.edges(ctx.stats().get('n_edges', 0))
    np.save(os.path.join(out_dir, f'edges{rank}.npy'), np.stack([a, b, I, U], axis=1) if len(a) else np.zeros((0, 4)))
    np.save(os.path.join(out_dir, f'info{rank}.npy'), np.array([info['capped'], info['max_fwd']]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize('edge_threshold', [10, 2])
def test_gloo_world2_sweep_shard_equals_oracle(world_case, tmp_path, edge_threshold):
    """dist.SweepShard over gloo with world_size 2 (real all_to_all of entries, all-reduce of the
    forward degree, all-gather of labels) on the emulated device: both ranks end with the oracle's
    components; the ranks' edges partition the oracle's edges.  edge_threshold 2 makes the cap bind:
    the sharded replay's exchanges run for real (gathered E* rows, the local T-T forests, the hit lists
    to the components' ranks — the emulator checks each rank's assembled lists against an unfiltered
    index — and the change lists) and the ranks' capped edges partition the oracle's capped graph."""
    import torch.multiprocessing as mp
    from fslr_amd.prep import fold_overlap_threshold
    csr, o = world_case
    thr = fold_overlap_threshold(csr.iv_aln, 0.8)
    mp.start_processes(_sweep_worker, args=(2, _free_port(), csr, thr, str(tmp_path), edge_threshold), nprocs=2,
                       join=True, start_method='spawn')
    oc = _oracle_csr(csr)
    ref = o if edge_threshold == 10 else O.run_core(oc, use_cap=True, edge_threshold=edge_threshold)
    capped = [bool(np.load(tmp_path / f'info{r}.npy')[0]) for r in range(2)]
    assert capped[0] == capped[1] == (int(o['fwd'].max()) > edge_threshold)     # o: uncapped E*
    assert capped[0] == (edge_threshold == 2)
    for r in range(2):
        got = np.load(tmp_path / f'labels{r}.npy')
        np.testing.assert_array_equal(_components_from_labels(got), ref['comp'])
    if not capped[0]:
        e = np.concatenate([np.load(tmp_path / f'edges{r}.npy') for r in range(2)]).astype(np.int64)
        got = sorted(map(tuple, e.tolist()))
        want = sorted(zip(o['edge_a'].tolist(), o['edge_b'].tolist(), o['edge_I'].tolist(), o['edge_U'].tolist()))
        assert got == want
    else:
        # the sharded replay: the ranks' capped edges (re-oriented as (former, partner)) partition the
        # oracle's capped graph
        want = sorted(zip(ref['edge_a'].tolist(), ref['edge_b'].tolist(), ref['edge_I'].tolist(),
                          ref['edge_U'].tolist()))
        e = np.concatenate([np.load(tmp_path / f'edges{r}.npy') for r in range(2)]).astype(np.int64)
        assert sorted(map(tuple, e.tolist())) == want


@pytest.mark.parametrize('edge_threshold,gather', [(10, 'restricted'), (2, 'restricted'), (2, 'full'), (2, 'i32')])
def test_local_hub_w3_sweep_shard_equals_oracle(world_case, edge_threshold, gather, monkeypatch):
    """dist.SweepShard on W = 3 ranks as threads over dist.LocalHub (the in-process collectives the
    10M-read GPU test runs the product split with), on the emulated device: every rank has the
    oracle's components and the ranks' edges partition the oracle's (capped when edge_threshold 2)."""
    import threading
    from fslr_amd.dist import LocalHub, SweepShard, chrom_counts_of
    from fslr_amd.prep import fold_overlap_threshold, pass_table
    from tests.sweep_emu import EmuSweepContext
    monkeypatch.setenv('FSLR_CAP_GATHER', 'full' if gather == 'full' else 'restricted')
    if gather == 'i32':
        monkeypatch.setenv('FSLR_CAP_BWD', 'i32')
    csr, o = world_case
    thr = fold_overlap_threshold(csr.iv_aln, 0.8)
    pt = pass_table([1, 1, 0.66, 0.66, 0.66, 0.5])
    W = 3
    hub = LocalHub(W, timeout=120)
    ctxs = [EmuSweepContext(csr, thr) for _ in range(W)]
    infos, errs = [None] * W, [None] * W

    def run(r):
        try:
            sh = SweepShard(ctxs[r], csr.n_reads, chrom_counts_of(csr), W, r, 'cpu', comm=hub.comm(r, 'cpu'))
            infos[r] = sh.step(1 - 0.04, 1 - 0.25, pt, edge_threshold)
        except BaseException as e:                     # noqa: BLE001
            errs[r] = e
            hub.barrier.abort()

    ts = [threading.Thread(target=run, args=(r,)) for r in range(W)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    for e in errs:
        if e is not None:
            raise e
    ref = o if edge_threshold == 10 else O.run_core(_oracle_csr(csr), use_cap=True, edge_threshold=edge_threshold)
    assert all(i['capped'] == (edge_threshold == 2) for i in infos)
    if edge_threshold == 2:
        assert all(i['cap']['max_fwd'] == int(ref['fwd'].max()) for i in infos)
    got = []
    for c in ctxs:
        a, b, I, U = c.edges(c.stats()['n_edges'])
        got += list(zip(a.tolist(), b.tolist(), I.tolist(), U.tolist()))
        np.testing.assert_array_equal(_components_from_labels(c.labels()), ref['comp'])
    want = sorted(zip(ref['edge_a'].tolist(), ref['edge_b'].tolist(), ref['edge_I'].tolist(), ref['edge_U'].tolist()))
    assert sorted(got) == want


def _one_stream():
    """One non-default torch stream, made current and shared with every context of a test: the
    in-process 'collectives' (torch.cat of device buffers) then run in order with the kernels that
    write and read those buffers (each context otherwise owns a stream of its own)."""
    import torch
    s = torch.cuda.Stream(torch.device('cuda', 0))
    torch.cuda.set_stream(s)
    return s


def _sweep_split_on_device(csr, thr, pt, W, edge_threshold=10, block_shift=6):
    """Run the chromosome split with W contexts on cuda:0, the exchange done in-process (the
    concatenation of every rank's segment for each destination).  Returns the contexts (their
    edges and labels after the in-process label merge) and the per-rank entry counts."""
    import torch
    from fslr_amd import _lib
    from fslr_amd.dist import chrom_counts_of, chrom_owner
    dev = torch.device('cuda', 0)
    stream = _one_stream()                         # torch's copies and the contexts' kernels in order
    owner = chrom_owner(chrom_counts_of(csr), W)
    segs = [[] for _ in range(W)]
    sent = []
    for r in range(W):
        c = _lib.Context(0, stream=stream.cuda_stream)
        c.load_csr(csr, thr)
        c.set_chrom_filter(owner == r)
        c.build_index()
        buf = torch.empty(1 << 16, dtype=torch.int64, device=dev)
        ok, counts = c.sweep_partition(1 - 0.04, 1 - 0.25, pt, W, block_shift, buf)
        if not ok:
            buf = torch.empty(int(counts.sum()) + 16, dtype=torch.int64, device=dev)
            ok, counts = c.sweep_partition(1 - 0.04, 1 - 0.25, pt, W, block_shift, buf)
        assert ok
        pos = np.concatenate([[0], np.cumsum(counts)])
        for d in range(W):
            segs[d].append(buf[pos[d]:pos[d + 1]].clone())
        sent.append(counts)
        c.close()
    ctxs = []
    for d in range(W):
        c = _lib.Context(0, stream=stream.cuda_stream)
        c.load_csr(csr, thr)
        c.reserve_edges(12 * csr.n_reads)
        ent = torch.cat(segs[d]) if segs[d] else torch.empty(0, dtype=torch.int64, device=dev)
        c.sweep_evaluate(1 - 0.04, 1 - 0.25, pt, ent, ent.numel(), edge_threshold)
        torch.cuda.synchronize()
        c.components()
        ctxs.append(c)
    n = csr.n_reads
    locals_ = []
    for c in ctxs:
        t = torch.empty(n, dtype=torch.int32, device=dev)
        c.labels_into(t)
        locals_.append(t)
    torch.cuda.synchronize()
    gathered = torch.cat(locals_)
    for c in ctxs:
        c.union_label_vectors(gathered)
    torch.cuda.synchronize()
    return ctxs, np.array(sent)


@pytest.mark.gpu
@pytest.mark.parametrize('W', [2, 3, 8])
def test_sweep_split_contexts_one_gpu_equals_oracle(W):
    """fslr_set_chrom_filter / fslr_sweep_partition / fslr_sweep_evaluate with W contexts on one
    GPU: the destinations' edges (a, b, I, U) partition the oracle's edges, their forward degrees
    add up to the oracle's, and after the label merge every context has the oracle's components."""
    from fslr_amd.dist import shard_of
    from fslr_amd.prep import fold_overlap_threshold, pass_table
    s = synth.generate(40_000, 16, 21)
    csr = s.interval_data().csr()
    thr = fold_overlap_threshold(csr.iv_aln, 0.8)
    pt = pass_table([1, 1, 0.66, 0.66, 0.66, 0.5])
    o = O.run_core(_oracle_csr(csr), use_cap=False)
    ctxs, sent = _sweep_split_on_device(csr, thr, pt, W)
    want = sorted(zip(o['edge_a'].tolist(), o['edge_b'].tolist(), o['edge_I'].tolist(), o['edge_U'].tolist()))
    got = []
    fwd = np.zeros(csr.n_reads, np.int64)
    for d, c in enumerate(ctxs):
        st = c.stats()
        a, b, I, U = c.edges(st['n_edges'])
        assert (shard_of(a, W) == d).all()           # 64-rank blocks round robin, as shard_of
        got += list(zip(a.tolist(), b.tolist(), I.tolist(), U.tolist()))
        fwd += c.fwd_degree()
    assert sorted(got) == want
    np.testing.assert_array_equal(fwd, o['fwd'])
    for c in ctxs:
        np.testing.assert_array_equal(_components_from_labels(c.labels()), o['comp'])
        c.close()
    # every rank sent something and the chromosome split is roughly balanced
    per_rank = sent.sum(axis=1)
    assert per_rank.min() > 0 and per_rank.max() < 2.0 * per_rank.mean()


def _sweep_shards_threads(csr, thr, pt, W, edge_threshold, steps=1, split='chrom'):
    """The product's dist.SweepShard on W ranks that are threads of this process, each with its own
    context and stream on cuda:0, the collectives in-process (dist.LocalHub: a device synchronize,
    then every rank copies what it needs).  Returns (contexts, step infos of the last step)."""
    import threading
    import torch
    from fslr_amd import _lib
    from fslr_amd.dist import LocalHub, SweepShard, chrom_counts_of
    dev = torch.device('cuda', 0)
    hub = LocalHub(W)
    ctxs, infos, errs = [None] * W, [None] * W, [None] * W

    def run(r):
        try:
            s = torch.cuda.Stream(dev)
            torch.cuda.set_stream(s)
            c = _lib.Context(0, stream=s.cuda_stream)
            ctxs[r] = c
            c.load_csr(csr, thr)
            c.reserve_edges(max(1 << 16, 12 * csr.n_reads // W))
            sh = SweepShard(c, csr.n_reads, chrom_counts_of(csr), W, r, dev, comm=hub.comm(r, dev), split=split)
            for _ in range(steps):
                infos[r] = sh.step(1 - 0.04, 1 - 0.25, pt, edge_threshold)
            infos[r]['pos'] = sh.pos
            torch.cuda.synchronize(dev)
        except BaseException as e:                     # noqa: BLE001 - re-raised by the caller
            errs[r] = e
            hub.barrier.abort()

    ts = [threading.Thread(target=run, args=(r,)) for r in range(W)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    for e in errs:
        if e is not None and not isinstance(e, threading.BrokenBarrierError):
            raise e
    for e in errs:
        if e is not None:
            raise e
    return ctxs, infos


def _union_view(ctxs):
    """The ranks' edges (a, b, I, U) concatenated and their forward degrees summed."""
    parts = [c.edges(c.stats()['n_edges']) for c in ctxs]
    a, b, I, U = (np.concatenate([p[k] for p in parts]) for k in range(4))
    fwd = np.sum([c.fwd_degree().astype(np.int64) for c in ctxs], axis=0)
    return a, b, I, U, fwd


@pytest.mark.gpu
@pytest.mark.parametrize('W,thr,gather', [(1, 3, 'restricted'), (2, 3, 'restricted'), (8, 3, 'restricted'),
                                          (1, 10, 'restricted'), (2, 10, 'restricted'), (8, 10, 'restricted'),
                                          (2, 3, 'full'), (8, 10, 'full'), (2, 3, 'i32'), (8, 3, 'i32')])
def test_sweep_split_capped_one_gpu_equals_oracle(W, thr, gather, monkeypatch):
    """The product's SweepShard with a binding cap, W ranks as threads on one GPU: the sharded replay
    (each rank lists the hits of its chromosomes, the lists travel to the rank replaying their read's
    component, the changes are exchanged) on a dense input where the cap binds for many reads — the
    ranks' capped edges (as (former, partner, I, U)) are the oracle's reference loop's, their edges
    per loop add up to the oracle's, and every rank has the oracle's components.  ``gather``: the
    rows of S only (uint8 or int32 backward counts summed over the ranks), or every E* row."""
    import dataclasses
    monkeypatch.setenv('FSLR_CAP_GATHER', 'full' if gather == 'full' else 'restricted')
    if gather == 'i32':
        monkeypatch.setenv('FSLR_CAP_BWD', 'i32')
    from fslr_amd.prep import fold_overlap_threshold, pass_table
    s = synth.generate(20_000, 16, 47, cluster_cap=30, size_p=0.05)
    csr = s.interval_data().csr()
    st = csr.iv_start.astype(np.int64) // 100
    en = st + (csr.iv_end.astype(np.int64) - csr.iv_start)
    csr = dataclasses.replace(csr, iv_start=st.astype(np.int32), iv_end=en.astype(np.int32))
    thr_iv = fold_overlap_threshold(csr.iv_aln, 0.8)
    pt = pass_table([1, 1, 0.66, 0.66, 0.66, 0.5])
    o = O.run_core(_oracle_csr(csr), edge_threshold=thr, use_cap=True)
    ctxs, infos = _sweep_shards_threads(csr, thr_iv, pt, W, thr, steps=2)
    try:
        assert all(i['capped'] for i in infos)
        caps = [i['cap'] for i in infos]
        assert all(cp == caps[0] for cp in caps)
        assert caps[0]['capped'] > 0 and caps[0]['dropped'] > 0
        assert caps[0]['max_fwd'] == int(o['fwd'].max())
        want = sorted(zip(o['edge_a'].tolist(), o['edge_b'].tolist(), o['edge_I'].tolist(), o['edge_U'].tolist()))
        a, b, I, U, fwd = _union_view(ctxs)
        assert sorted(zip(a.tolist(), b.tolist(), I.tolist(), U.tolist())) == want
        np.testing.assert_array_equal(fwd, o['fwd'])
        for c in ctxs:
            np.testing.assert_array_equal(_components_from_labels(c.labels()), o['comp'])
    finally:
        for c in ctxs:
            c.close()


def _zd_overflow_csr(n_dense=60, n_zd=400, seed=5):
    """A dense locus where the cap binds (n_dense reads) beside a locus of n_zd reads with qlen2 == 0,
    whose pairs all raise ZeroDivisionError (cluster.py:178-183): n_zd (n_zd - 1) / 2 listed pairs, more
    than the list's first capacity (65,536)."""
    from fslr_amd.prep import IntervalData
    rng = np.random.default_rng(seed)
    n = n_dense + n_zd
    start = np.concatenate([100_000 + rng.integers(0, 40, n_dense), 900_000 + rng.integers(0, 40, n_zd)])
    size = np.full(n, 1000)
    qlen2 = np.concatenate([np.full(n_dense, 3000), np.zeros(n_zd, np.int64)])
    o = np.argsort(start, kind='quicksort')
    col = lambda x: np.asarray(x, np.int64)[o]
    d = IntervalData(chrom=np.ones(n, np.int64)[o], start=col(start), end=col(start + size), aln_size=col(size),
                     qcode=col(np.arange(n)), qnames=np.array([f'r{k}' for k in range(n)], dtype=object),
                     n_alignments=np.full(n, 2, np.int64), qlen2=col(qlen2), middle=np.zeros(n, np.int64),
                     index=np.arange(n))
    return d.csr()


@pytest.mark.gpu
@pytest.mark.parametrize('W', [1, 2])
def test_sweep_split_zero_division_list_overflow_follows_oracle(W):
    """More ZeroDivisionError pairs than the device list holds, with the cap binding: the partition
    (a zd_host query) grows the list and runs again, so the sharded replay decides on every pair and the
    step raises like the oracle's reference loop — not 'rerun the query' forever."""
    from fslr_amd.prep import fold_overlap_threshold, pass_table
    csr = _zd_overflow_csr()
    pt = pass_table([1, 1, 0.66, 0.66, 0.66, 0.5])
    try:
        o = O.run_core(_oracle_csr(csr), edge_threshold=10, use_cap=True)
    except O.OracleZeroDivision:
        o = None
    thr_iv = fold_overlap_threshold(csr.iv_aln, 0.8)
    if o is None:
        with pytest.raises(ZeroDivisionError):
            _sweep_shards_threads(csr, thr_iv, pt, W, 10)
        return
    ctxs, infos = _sweep_shards_threads(csr, thr_iv, pt, W, 10)
    try:
        a, b, I, U, fwd = _union_view(ctxs)
        want = sorted(zip(o['edge_a'].tolist(), o['edge_b'].tolist(), o['edge_I'].tolist(), o['edge_U'].tolist()))
        assert sorted(zip(a.tolist(), b.tolist(), I.tolist(), U.tolist())) == want
    finally:
        for c in ctxs:
            c.close()


def _sweep_gpu_worker(rank, world, port, out_dir):
    import torch
    import torch.distributed as dist
    from fslr_amd import _lib
    from fslr_amd.dist import SweepShard, chrom_counts_of
    from fslr_amd.prep import fold_overlap_threshold, pass_table
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    s = synth.generate(40_000, 16, 21)
    csr = s.interval_data().csr()
    dev = torch.device('cuda', 0)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    ctx = _lib.Context(0, stream=stream.cuda_stream)
    ctx.load_csr(csr, fold_overlap_threshold(csr.iv_aln, 0.8))
    sh = SweepShard(ctx, csr.n_reads, chrom_counts_of(csr), world, rank, dev)
    pt = pass_table([1, 1, 0.66, 0.66, 0.66, 0.5])
    for _ in range(2):                               # the second step reuses the grown buffers
        info = sh.step(1 - 0.04, 1 - 0.25, pt, 10)
    info = sh.step(1 - 0.04, 1 - 0.25, pt, 10, repeat=True)     # as bench.py's timed steps
    assert info.get('repeat')
    sh.verify_repeat()
    np.save(os.path.join(out_dir, f'labels{rank}.npy'), sh.labels())
    st = ctx.stats()
    a, b, I, U = ctx.edges(st['n_edges'])
    np.save(os.path.join(out_dir, f'edges{rank}.npy'), np.stack([a, b, I, U], axis=1))
    np.save(os.path.join(out_dir, f'info{rank}.npy'), np.array([info['capped'], info['entries_sent']]))
    dist.barrier()
    ctx.close()
    dist.destroy_process_group()


@pytest.mark.gpu
def test_sweep_shard_gloo_two_processes_one_gpu(tmp_path):
    """dist.SweepShard as bench.py runs it, two processes sharing cuda:0 over gloo (entries and
    labels staged through host memory): edges partition the oracle's, labels are the oracle's."""
    import torch.multiprocessing as mp
    mp.start_processes(_sweep_gpu_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True,
                       start_method='spawn')
    s = synth.generate(40_000, 16, 21)
    csr = s.interval_data().csr()
    o = O.run_core(_oracle_csr(csr), use_cap=False)
    e = np.concatenate([np.load(tmp_path / f'edges{r}.npy') for r in range(2)]).astype(np.int64)
    want = sorted(zip(o['edge_a'].tolist(), o['edge_b'].tolist(), o['edge_I'].tolist(), o['edge_U'].tolist()))
    assert sorted(map(tuple, e.tolist())) == want
    for r in range(2):
        np.testing.assert_array_equal(_components_from_labels(np.load(tmp_path / f'labels{r}.npy')), o['comp'])
        assert not np.load(tmp_path / f'info{r}.npy')[0]


def _sweep_gpu_tamper_worker(rank, world, port, out_dir):
    import torch
    import torch.distributed as dist
    from fslr_amd import _lib
    from fslr_amd.dist import SweepShard, chrom_counts_of
    from fslr_amd.prep import fold_overlap_threshold, pass_table
    # capi.hip: ablation bit 64 makes fslr_sweep_partition_repeat expect one entry more for
    # destination 0 than the synchronous partition wrote, as a partition that landed differently would
    os.environ['FSLR_ABLATE'] = '64' if rank == 1 else '0'
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    s = synth.generate(20_000, 16, 23)
    csr = s.interval_data().csr()
    dev = torch.device('cuda', 0)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    ctx = _lib.Context(0, stream=stream.cuda_stream)
    ctx.load_csr(csr, fold_overlap_threshold(csr.iv_aln, 0.8))
    sh = SweepShard(ctx, csr.n_reads, chrom_counts_of(csr), world, rank, dev)
    pt = pass_table([1, 1, 0.66, 0.66, 0.66, 0.5])
    sh.step(1 - 0.04, 1 - 0.25, pt, 10)
    info = sh.step(1 - 0.04, 1 - 0.25, pt, 10, repeat=True)
    assert info.get('repeat')
    raised = 0
    try:
        sh.verify_repeat()
    except _lib.FslrError:
        raised = 1
    np.save(os.path.join(out_dir, f'raised{rank}.npy'), np.array([raised]))
    # a synchronous step starts a new series: clean again
    sh.step(1 - 0.04, 1 - 0.25, pt, 10)
    assert not ctx.stats()['overflow_flags'] & 32
    dist.barrier()
    ctx.close()
    dist.destroy_process_group()


@pytest.mark.gpu
def test_sweep_shard_repeat_mismatch_raises_on_every_rank(tmp_path):
    """A repeat step whose device partition differs from the synchronous step's (forced on rank 1)
    is caught by verify_repeat() on both ranks: the flag survives the evaluation that follows the
    partition (round-3 advice: the per-query reset used to erase it)."""
    import torch.multiprocessing as mp
    mp.start_processes(_sweep_gpu_tamper_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True,
                       start_method='spawn')
    for r in range(2):
        assert int(np.load(tmp_path / f'raised{r}.npy')[0]) == 1


def test_multi_csr_handoff_roundtrip(tmp_path, world_case):
    """fslr_amd.multi hands the prepared CSR to the rank processes as .npy files: every field the
    ranks upload comes back unchanged, with the query parameters."""
    from fslr_amd import multi
    from fslr_amd.prep import fold_overlap_threshold, pass_table
    csr, _ = world_case
    thr = fold_overlap_threshold(csr.iv_aln, 0.8)
    pt = pass_table([1, 1, 0.66])
    multi._save(str(tmp_path), csr, thr, dict(qlen_cut=0.96, nal_cut=0.75, pass_table=pt, edge_threshold=10))
    c2, thr2, pt2, meta = multi._load(str(tmp_path))
    for f in multi._CSR_FIELDS:
        np.testing.assert_array_equal(np.asarray(getattr(c2, f)), np.asarray(getattr(csr, f)))
    np.testing.assert_array_equal(thr2, thr)
    np.testing.assert_array_equal(pt2, pt)
    assert c2.n_chroms == csr.n_chroms and meta['edge_threshold'] == 10 and meta['qlen_cut'] == 0.96
    assert multi.sweep_applies(csr, thr)
    assert not multi.sweep_applies(csr, fold_overlap_threshold(csr.iv_aln, 0.0))


def test_cli_exposes_gpus_option():
    from click.testing import CliRunner
    from fslr_amd.main import pipeline
    out = CliRunner().invoke(pipeline, ['--help']).output
    assert '--gpus' in out


def _sweep_zerodiv_worker(rank, world, port, csr, thr, out_dir):
    import torch.distributed as dist
    from fslr_amd.dist import SweepShard, chrom_counts_of
    from fslr_amd.prep import pass_table
    from tests.sweep_emu import EmuSweepContext
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    ctx = EmuSweepContext(csr, thr)
    sh = SweepShard(ctx, csr.n_reads, chrom_counts_of(csr), world, rank, 'cpu')
    raised = ''
    try:
        sh.step(1 - 0.04, 1 - 0.25, pass_table([1, 1, 0.66, 0.66, 0.66, 0.5]), 10)
    except ZeroDivisionError as e:
        raised = f'ZeroDivisionError: {e}'
    with open(os.path.join(out_dir, f'raised{rank}.txt'), 'w') as fh:
        fh.write(raised)
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_zero_division_raises_on_every_rank(world_case, tmp_path):
    """The reference raises ZeroDivisionError when both reads of a candidate pair have qlen2 0
    (cluster.py:178-183).  Only the rank that sweeps that pair's chromosome sees it; the negative
    count it sends in the counts exchange makes every rank raise instead of waiting in a collective."""
    import dataclasses
    import torch.multiprocessing as mp
    from fslr_amd.prep import fold_overlap_threshold
    csr, o = world_case
    a, b = int(o['edge_a'][0]), int(o['edge_b'][0])
    q = np.array(csr.read_qlen2, copy=True)
    q[[a, b]] = 0
    bad = dataclasses.replace(csr, read_qlen2=q)
    thr = fold_overlap_threshold(bad.iv_aln, 0.8)
    mp.start_processes(_sweep_zerodiv_worker, args=(2, _free_port(), bad, thr, str(tmp_path)), nprocs=2,
                       join=True, start_method='spawn')
    for r in range(2):
        assert (tmp_path / f'raised{r}.txt').read_text().startswith('ZeroDivisionError')


@pytest.mark.gpu
def test_sweep_partition_first_call_in_reused_memory():
    """The first fslr_sweep_partition on a fresh context overflows its upper-bound slots (sized for
    4 pair tests per interval) and reruns; the grouping pass that runs before the overflow check must
    see every tile's count defined even when the context's buffers come from freed, dirty device
    memory (round-3 fix: a skipped tile's count was left unwritten)."""
    import torch
    from fslr_amd import _lib
    from fslr_amd.dist import chrom_counts_of, chrom_owner
    from fslr_amd.prep import fold_overlap_threshold, pass_table
    dirty = torch.full((1 << 28,), -1, dtype=torch.int32, device='cuda')      # 1 GiB of 0xFF bytes
    torch.cuda.synchronize()
    del dirty
    torch.cuda.empty_cache()                         # back to the HIP allocator, contents kept
    import dataclasses
    s = synth.generate(40_000, 16, 29)
    csr = s.interval_data().csr()
    st = csr.iv_start.astype(np.int64) // 50             # squeezed: ~2.8M pair tests per rank > 1M slots
    en = st + (csr.iv_end.astype(np.int64) - csr.iv_start)
    csr = dataclasses.replace(csr, iv_start=st.astype(np.int32), iv_end=en.astype(np.int32))
    thr = fold_overlap_threshold(csr.iv_aln, 0.8)
    pt = pass_table([1, 1, 0.66, 0.66, 0.66, 0.5])
    o = O.run_core(_oracle_csr(csr), use_cap=False)
    ctxs, _ = _sweep_split_on_device(csr, thr, pt, 2)
    got = []
    for c in ctxs:
        a, b, I, U = c.edges(c.stats()['n_edges'])
        got += list(zip(a.tolist(), b.tolist(), I.tolist(), U.tolist()))
        c.close()
    assert sorted(got) == sorted(zip(o['edge_a'].tolist(), o['edge_b'].tolist(), o['edge_I'].tolist(),
                                     o['edge_U'].tolist()))


@pytest.mark.gpu
def test_sweep_partition_repeat_equals_sync():
    """fslr_sweep_partition_repeat (the timed multi-GPU steps of bench.py): on unchanged input it
    writes each destination's segment with the same entries as the synchronous partition, with no
    flag raised; another split or a new input generation is refused."""
    import torch
    from fslr_amd import _lib
    from fslr_amd.dist import chrom_counts_of, chrom_owner
    from fslr_amd.prep import fold_overlap_threshold, pass_table
    s = synth.generate(20_000, 16, 5)
    csr = s.interval_data().csr()
    thr = fold_overlap_threshold(csr.iv_aln, 0.8)
    pt = pass_table([1, 1, 0.66, 0.66, 0.66, 0.5])
    qc, nc = 1 - 0.04, 1 - 0.25
    ctx = _lib.Context(0)
    ctx.load_csr(csr, thr)
    ctx.set_chrom_filter(chrom_owner(chrom_counts_of(csr), 2) == 0)
    ctx.build_index()
    dst = torch.empty(1 << 16, dtype=torch.int64, device='cuda')
    ok, counts = ctx.sweep_partition(qc, nc, pt, 3, 6, dst)
    if not ok:
        dst = torch.empty(int(counts.sum()) + 4096, dtype=torch.int64, device='cuda')
        ok, counts = ctx.sweep_partition(qc, nc, pt, 3, 6, dst)
    assert ok and counts.sum() > 0
    pos = np.concatenate([[0], np.cumsum(counts)])
    ref = dst[:pos[-1]].cpu().numpy()
    dst.fill_(0)
    torch.cuda.synchronize()
    for _ in range(2):
        ctx.build_index()
        ctx.sweep_partition_repeat(qc, nc, pt, 3, 6, dst)
        ctx.sync()
        got = dst[:pos[-1]].cpu().numpy()
        for d in range(3):                       # order inside a segment is free (LDS atomics)
            np.testing.assert_array_equal(np.sort(got[pos[d]:pos[d + 1]]), np.sort(ref[pos[d]:pos[d + 1]]))
        st = ctx.stats()
        assert not st['overflow_flags'] & 32
    with pytest.raises(_lib.FslrError):
        ctx.sweep_partition_repeat(qc, nc, pt, 2, 6, dst)          # another split
    ctx.set_thresholds(thr)                                        # a new input generation
    ctx.set_chrom_filter(chrom_owner(chrom_counts_of(csr), 2) == 0)
    ctx.build_index()
    with pytest.raises(_lib.FslrError):
        ctx.sweep_partition_repeat(qc, nc, pt, 3, 6, dst)
    ctx.close()


def skewed_case(n=6000, seed=37):
    """>= 50 % of the intervals on one chromosome (a targeted-panel genome): the chromosome split cannot
    balance it, the position split can."""
    w = np.ones(len(synth.CHROMS))
    w[0] = len(synth.CHROMS) * 1.2
    s = synth.generate(n, 8, seed, chrom_weights=w)
    return s.interval_data().csr()


def test_position_plan_balances_a_skewed_genome():
    """position_plan cuts the sorted positions where the emulated pair tests balance; the ranges tile the
    index, every range holds its forward windows, and the most loaded rank is within 1.2 of the mean
    (the chromosome split: > 3 x at W = 8)."""
    from fslr_amd.dist import chrom_owner, position_plan
    from fslr_amd.prep import fold_overlap_threshold
    from tests.sweep_emu import EmuSweepContext
    csr = skewed_case(20000)
    counts = np.bincount(csr.iv_chrom, minlength=csr.n_chroms)
    assert counts.max() >= 0.5 * counts.sum()
    ctx = EmuSweepContext(csr, fold_overlap_threshold(csr.iv_aln, 0.8))
    tests, reach = ctx.position_costs()
    nf = ctx._n_fwd()
    cost = nf + 4
    for W in (2, 4, 8):
        plan = position_plan(tests, reach, csr.n_intervals, W)
        assert plan[0][0] == 0 and plan[-1][1] == csr.n_intervals
        for (a0, a1, e), (b0, _, _) in zip(plan, plan[1:]):
            assert a1 == b0
        for lo, hi, end in plan:
            q = np.arange(lo, hi)
            assert (q + nf[lo:hi] < end).all() and end <= csr.n_intervals
        per = np.array([cost[lo:hi].sum() for lo, hi, _ in plan])
        assert per.max() <= 1.2 * per.mean() + 64 * 40, (W, per)
        own = chrom_owner(counts, W)
        pos_c = np.asarray(csr.iv_chrom)[np.argsort(ctx.pos)]
        per_c = np.array([cost[np.isin(pos_c, np.flatnonzero(own == r))].sum() for r in range(W)])
        if W == 8:
            assert per_c.max() > 3 * per_c.mean()


def _pos_worker(rank, world, port, csr, thr, out_dir, edge_threshold):
    import torch.distributed as dist
    from fslr_amd.dist import SweepShard, chrom_counts_of
    from fslr_amd.prep import pass_table
    from tests.sweep_emu import EmuSweepContext
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    ctx = EmuSweepContext(csr, thr)
    sh = SweepShard(ctx, csr.n_reads, chrom_counts_of(csr), world, rank, 'cpu', split='position')
    pt = pass_table([1, 1, 0.66, 0.66, 0.66, 0.5])
    info = sh.step(1 - 0.04, 1 - 0.25, pt, edge_threshold)
    info2 = sh.step(1 - 0.04, 1 - 0.25, pt, edge_threshold, repeat=True)
    assert info2.get('repeat', False) == (not info['capped'])
    np.save(os.path.join(out_dir, f'labels{rank}.npy'), sh.labels())
    a, b, I, U = ctx.edges(ctx.stats().get('n_edges', 0))
    np.save(os.path.join(out_dir, f'edges{rank}.npy'), np.stack([a, b, I, U], axis=1) if len(a) else np.zeros((0, 4)))
    np.save(os.path.join(out_dir, f'pos{rank}.npy'), np.array(sh.pos))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize('edge_threshold', [10, 2])
def test_gloo_world2_position_split_equals_oracle(tmp_path, edge_threshold):
    """SweepShard(split='position') over gloo at world size 2 on a skewed genome: the ranks' ranges tile
    the sorted positions (one chromosome spans both), the ranks' edges partition the oracle's (capped
    with edge_threshold 2: the replay lists its hits on the chromosome split) and every rank has the
    oracle's components."""
    import torch.multiprocessing as mp
    from fslr_amd.prep import fold_overlap_threshold
    csr = skewed_case()
    thr = fold_overlap_threshold(csr.iv_aln, 0.8)
    mp.start_processes(_pos_worker, args=(2, _free_port(), csr, thr, str(tmp_path), edge_threshold), nprocs=2,
                       join=True, start_method='spawn')
    ref = O.run_core(_oracle_csr(csr), use_cap=True, edge_threshold=edge_threshold)
    p0, p1 = np.load(tmp_path / 'pos0.npy'), np.load(tmp_path / 'pos1.npy')
    assert p0[0] == 0 and p0[1] == p1[0] and p1[1] == csr.n_intervals
    for r in range(2):
        np.testing.assert_array_equal(_components_from_labels(np.load(tmp_path / f'labels{r}.npy')), ref['comp'])
    e = np.concatenate([np.load(tmp_path / f'edges{r}.npy') for r in range(2)]).astype(np.int64)
    want = sorted(zip(ref['edge_a'].tolist(), ref['edge_b'].tolist(), ref['edge_I'].tolist(), ref['edge_U'].tolist()))
    assert sorted(map(tuple, e.tolist())) == want


@pytest.mark.gpu
@pytest.mark.parametrize('W,edge_threshold', [(8, 10), (8, 3), (3, 10)])
def test_position_split_skewed_genome_one_gpu_equals_oracle(W, edge_threshold):
    """A genome with >= 50 % of the intervals on one chromosome through the product's
    SweepShard(split='position') at W ranks (threads on one GPU): the ranges tile the sorted positions
    and split that chromosome, the ranks' edges partition the oracle's (capped at 3: the replay's hit
    lists come from the chromosome split), every rank has the oracle's components; two steps each."""
    from fslr_amd.prep import fold_overlap_threshold, pass_table
    w = np.ones(len(synth.CHROMS))
    w[0] = len(synth.CHROMS) * 1.2
    s = synth.generate(150_000, 16, 53, chrom_weights=w)
    csr = s.interval_data().csr()
    counts = np.bincount(csr.iv_chrom, minlength=csr.n_chroms)
    assert counts.max() >= 0.5 * counts.sum()
    thr_iv = fold_overlap_threshold(csr.iv_aln, 0.8)
    pt = pass_table([1, 1, 0.66, 0.66, 0.66, 0.5])
    o = O.run_core(_oracle_csr(csr), edge_threshold=edge_threshold, use_cap=True)
    ctxs, infos = _sweep_shards_threads(csr, thr_iv, pt, W, edge_threshold, steps=2, split='position')
    try:
        pos = [i['pos'] for i in infos]
        assert pos[0][0] == 0 and pos[-1][1] == csr.n_intervals
        assert all(a[1] == b[0] for a, b in zip(pos, pos[1:]))
        h = int(np.argmax(counts))                # the heavy chromosome's sorted positions [big0, big1)
        big0 = int(counts[:h].sum())
        big1 = big0 + int(counts[h])
        assert sum(1 for lo, hi, _ in pos if lo < big1 and hi > big0) >= 2, pos
        want = sorted(zip(o['edge_a'].tolist(), o['edge_b'].tolist(), o['edge_I'].tolist(), o['edge_U'].tolist()))
        a, b, I, U, fwd = _union_view(ctxs)
        assert sorted(zip(a.tolist(), b.tolist(), I.tolist(), U.tolist())) == want
        np.testing.assert_array_equal(fwd, o['fwd'])
        for c in ctxs:
            np.testing.assert_array_equal(_components_from_labels(c.labels()), o['comp'])
    finally:
        for c in ctxs:
            c.close()


def _pair_shards_threads(csr, thr, pt, W, edge_threshold, long_reads=False, cutoffs=None):
    """dist.PairShard (the query-shard split) on W ranks as threads of this process, each with its own
    context and stream on cuda:0 and the full index."""
    import threading
    import torch
    from fslr_amd import _lib
    from fslr_amd.dist import LocalHub, PairShard
    from fslr_amd.prep import FSLR_THR_ZERO_ALN, umax_table
    dev = torch.device('cuda', 0)
    hub = LocalHub(W)
    ctxs, shards, infos, errs = [None] * W, [None] * W, [None] * W, [None] * W

    def run(r):
        try:
            s = torch.cuda.Stream(dev)
            torch.cuda.set_stream(s)
            c = _lib.Context(0, stream=s.cuda_stream)
            ctxs[r] = c
            if long_reads:
                c.load_csr_any(csr, np.where(np.asarray(csr.iv_aln) == 0, FSLR_THR_ZERO_ALN, 0))
                c.set_thresholds(thr)
                c.set_long_cutoffs(umax_table(cutoffs, int(np.diff(csr.read_off).max())))
            else:
                c.load_csr(csr, thr)
            c.reserve_edges(max(1 << 16, 12 * csr.n_reads))
            c.build_index()
            sh = shards[r] = PairShard(c, csr.n_reads, W, r, dev, comm=hub.comm(r, dev), long_reads=long_reads)
            infos[r] = sh.step(1 - 0.04, 1 - 0.25, pt, edge_threshold)
            torch.cuda.synchronize(dev)
        except BaseException as e:                     # noqa: BLE001 - re-raised by the caller
            errs[r] = e
            hub.barrier.abort()

    ts = [threading.Thread(target=run, args=(r,)) for r in range(W)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    for e in errs:
        if e is not None and not isinstance(e, threading.BrokenBarrierError):
            raise e
    for e in errs:
        if e is not None:
            raise e
    return ctxs, shards, infos


@pytest.mark.gpu
@pytest.mark.parametrize('case,W,edge_threshold', [('overlap0', 3, 10), ('overlap0', 2, 3), ('long', 3, 10),
                                                   ('long', 2, 3)])
def test_pair_shard_split_equals_oracle(case, W, edge_threshold):
    """The query-shard split (dist.PairShard) for the inputs the sweep split does not take — overlap 0
    (the walk engine's general thresholds) and reads of up to 150 intervals (the general evaluator,
    fslr_long_pairs_shard) — at W ranks (threads on one GPU):
    the ranks' parts of the edges and forward degrees add up to the oracle's graph (capped at 3: every
    rank replays the loops over the gathered E*), every rank has the oracle's components."""
    from fslr_amd.prep import fold_overlap_threshold, pass_table
    cut = [1, 1, 0.66, 0.66, 0.66, 0.5]
    overlap = 0.0 if case == 'overlap0' else 0.8
    if case == 'long':
        s = synth.generate(900, 150, 21, lmin=1)
    else:
        s = synth.generate(6000, 8, 29)
    csr = s.interval_data().csr()
    thr_iv = fold_overlap_threshold(csr.iv_aln, overlap)
    o = O.run_core(_oracle_csr(csr), overlap=overlap, edge_threshold=edge_threshold, use_cap=True)
    ctxs, shards, infos = _pair_shards_threads(csr, thr_iv, pass_table(cut), W, edge_threshold,
                                               long_reads=case == 'long', cutoffs=cut)
    try:
        assert all(i['path'] == ('long' if case == 'long' else 'walk') for i in infos)
        if edge_threshold == 3:
            assert all(i['capped'] for i in infos)
        a = np.concatenate([sh.edges_out[0] for sh in shards])
        b = np.concatenate([sh.edges_out[1] for sh in shards])
        I = np.concatenate([sh.edges_out[2] for sh in shards])
        U = np.concatenate([sh.edges_out[3] for sh in shards])
        want = sorted(zip(o['edge_a'].tolist(), o['edge_b'].tolist(), o['edge_I'].tolist(), o['edge_U'].tolist()))
        assert sorted(zip(a.tolist(), b.tolist(), I.tolist(), U.tolist())) == want
        np.testing.assert_array_equal(np.sum([sh.fwd_out.astype(np.int64) for sh in shards], axis=0), o['fwd'])
        for sh in shards:
            np.testing.assert_array_equal(_components_from_labels(sh.labels()), o['comp'])
    finally:
        for c in ctxs:
            if c is not None:
                c.close()
