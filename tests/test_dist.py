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
