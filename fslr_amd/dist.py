"""Multi-GPU sharding of the pair space (one process per GPU, torch.distributed over RCCL).

Partition: query reads are split into blocks of SHARD_BLOCK
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
