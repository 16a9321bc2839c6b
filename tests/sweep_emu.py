"""Host emulation of the sweep engine's multi-GPU entry points, for the CPU (gloo) tests of
fslr_amd.dist.SweepShard.  Test infrastructure only.

EmuSweepContext implements the Context methods SweepShard calls (fslr_hip.h
fslr_set_chrom_filter / fslr_sweep_partition / fslr_sweep_evaluate, components, the label
exchange) in numpy, with the device's entry encoding (a << 39 | b << 14 | i << 7 | j, a < b read
ranks, i / j interval slots in the reads) and its routing ((a >> shift) % n_dest).  It restates
what the kernels compute, not how; the device kernels are checked against the C oracle by the GPU
tests.  Here it lets the real torch.distributed exchange in dist.py run over gloo and be compared
with the oracle:
  * entries: every same-chromosome interval pair of two different reads whose overlap passes both
    intervals' folded thresholds (cluster.py:133-136, 159-160), for read pairs that pass the length
    gate (cluster.py:178-183);
  * evaluation: first-fit greedy over the pair's entries in (i, j) order (cluster.py:140-170),
    edge iff I > 0 and the cut table passes (cluster.py:216-219).
"""
from __future__ import annotations

import numpy as np

from fslr_amd.prep import FSLR_MAX_L, PASS_STRIDE


class EmuSweepContext:
    def __init__(self, csr, iv_thr, qlen_diff=0.04, n_aln_diff=0.25, overlap=0.8):
        self.csr = csr
        self.diffs = (qlen_diff, n_aln_diff, overlap)     # the cap replay hands these to the oracle
        self.thr = np.asarray(iv_thr, dtype=np.int64)
        assert (self.thr >= 1).all(), 'the sweep split needs overlap thresholds >= 1'
        self.n_reads = csr.n_reads
        off = np.asarray(csr.read_off, dtype=np.int64)
        self.read_of = np.repeat(np.arange(csr.n_reads), np.diff(off))
        self.slot = np.arange(off[-1]) - off[self.read_of]
        self.L = np.diff(off)
        self.owned = None
        self.edge_capacity = 1 << 30
        self._edges = np.zeros((0, 4), np.int64)
        self._parent = np.arange(self.n_reads)
        self._st = {}

    # -- filter / index ------------------------------------------------------------------------
    def set_chrom_filter(self, owned):
        self.owned = None if owned is None else np.asarray(owned, dtype=bool)

    def build_index(self):
        pass

    def reserve_edges(self, cap):
        pass

    # -- partition ------------------------------------------------------------------------------
    def _gate(self, a, b, qcut, ncut):
        q1, q2 = int(self.csr.read_qlen2[a]), int(self.csr.read_qlen2[b])
        mn, mx = min(q1, q2), max(q1, q2)
        if mx == 0:
            raise ZeroDivisionError('division by zero')
        if mn / mx >= qcut:
            return True
        n1, n2 = int(self.csr.read_nal[a]), int(self.csr.read_nal[b])
        mn, mx = min(n1, n2), max(n1, n2)
        if mx == 0:
            raise ZeroDivisionError('division by zero')
        return mn / mx >= ncut

    def _entries(self, qcut, ncut):
        c = self.csr
        chrom = np.asarray(c.iv_chrom)
        start, end = np.asarray(c.iv_start, np.int64), np.asarray(c.iv_end, np.int64)
        out = []
        for ch in np.unique(chrom):
            if self.owned is not None and not self.owned[ch]:
                continue
            ks = np.flatnonzero(chrom == ch)
            s, e = start[ks], end[ks]
            o = np.minimum(e[:, None], e[None, :]) - np.maximum(s[:, None], s[None, :])
            ok = (o >= self.thr[ks][:, None]) & (o >= self.thr[ks][None, :])
            ra, rb = self.read_of[ks][:, None], self.read_of[ks][None, :]
            ok &= ra < rb
            x, y = np.nonzero(ok)
            for p, q in zip(ks[x].tolist(), ks[y].tolist()):
                a, b = int(self.read_of[p]), int(self.read_of[q])
                if self._gate(a, b, qcut, ncut):
                    out.append((a << 39) | (b << 14) | (int(self.slot[p]) << 7) | int(self.slot[q]))
        return np.array(out, dtype=np.int64)

    def sweep_partition(self, qlen_cut, nal_cut, pass_table, n_dest, block_shift, dst, edge_threshold=10):
        ent = self._entries(qlen_cut, nal_cut)
        dest = (ent >> (39 + block_shift)) % n_dest
        order = np.argsort(dest, kind='stable')
        counts = np.bincount(dest, minlength=n_dest).astype(np.int64)
        if counts.sum() > dst.numel():
            return False, counts
        dst.numpy()[:ent.size] = ent[order]
        self._st = {'match_entries': int(ent.size)}
        return True, counts

    def sweep_partition_repeat(self, qlen_cut, nal_cut, pass_table, n_dest, block_shift, dst, edge_threshold=10):
        ok, counts = self.sweep_partition(qlen_cut, nal_cut, pass_table, n_dest, block_shift, dst, edge_threshold)
        assert ok, 'a repeat partition must fit where the synchronous one did'
        self.repeat_partitions = getattr(self, 'repeat_partitions', 0) + 1

    # -- evaluation -----------------------------------------------------------------------------
    def sweep_evaluate(self, qlen_cut, nal_cut, pass_table, entries, n, edge_threshold=10):
        ent = entries.numpy()[:n].astype(np.int64)
        pt = np.asarray(pass_table).reshape(FSLR_MAX_L, PASS_STRIDE)
        a = ent >> 39
        b = (ent >> 14) & 0x1FFFFFF
        i = (ent >> 7) & 127
        j = ent & 127
        order = np.lexsort((j, i, b, a))
        a, b, i, j = a[order], b[order], i[order], j[order]
        edges = []
        fwd = np.zeros(self.n_reads, np.int64)
        k = 0
        while k < a.size:
            m = k
            while m < a.size and a[m] == a[k] and b[m] == b[k]:
                m += 1
            used_i, used_j = set(), set()
            for t in range(k, m):                # (i, j) ascending: first free j for each i
                if i[t] in used_i or j[t] in used_j:
                    continue
                used_i.add(i[t])
                used_j.add(j[t])
            I = len(used_i)
            U = int(self.L[a[k]] + self.L[b[k]] - I)
            if I > 0 and pt[I - 1, U - 1]:
                edges.append((int(a[k]), int(b[k]), I, U))
                fwd[a[k]] += 1
            k = m
        self._edges = np.array(edges, dtype=np.int64).reshape(-1, 4)
        self._fwd = fwd
        self._st = {'n_edges': len(edges), 'edge_capacity': self.edge_capacity,
                    'max_fwd': int(fwd.max()) if fwd.size else 0}

    def stats(self, check=True):
        return dict(self._st)

    def edges(self, n_edges):
        e = self._edges[:n_edges]
        return e[:, 0], e[:, 1], e[:, 2], e[:, 3]

    def fwd_degree(self):
        return self._fwd.astype(np.int32)

    # -- components and the label exchange --------------------------------------------------------
    def _find(self, x):
        p = self._parent
        r = x
        while p[r] != r:
            r = p[r]
        while p[x] != r:
            p[x], x = r, p[x]
        return r

    def _union(self, x, y):
        rx, ry = self._find(x), self._find(y)
        if rx != ry:
            self._parent[max(rx, ry)] = min(rx, ry)

    def components(self):
        self._parent = np.arange(self.n_reads)
        for x, y in self._edges[:, :2].tolist():
            self._union(x, y)

    def labels(self):
        return np.array([self._find(v) for v in range(self.n_reads)], dtype=np.int32)

    def labels_into(self, t):
        t.numpy()[:] = self.labels()

    def edges_into(self, t, n_pad):
        e = self._edges[:n_pad]
        pairs = np.full((n_pad, 2), -1, dtype=np.int32)
        pairs[:len(e)] = e[:, :2]
        t.numpy()[:n_pad] = pairs.view(np.int64)[:, 0]

    def components_from_pairs(self, t, n):
        pairs = t.numpy()[:n].view(np.int32).reshape(-1, 2)
        self._parent = np.arange(self.n_reads)
        for x, y in pairs.tolist():
            if x >= 0:
                self._union(x, y)

    def union_label_vectors(self, t):
        lab = t.numpy()
        n = self.n_reads
        for k in range(lab.size):
            self._union(k % n, int(lab[k]))

    # -- the multi-GPU edge cap (fslr_cap_*): E* rows, candidates, search-ordered hit lists --------
    def edges_iu_into(self, t, n_pad):
        e = self._edges[:n_pad]
        rows = np.zeros((n_pad, 4), np.int32)
        rows[:, :2] = -1
        rows[:len(e), 0] = e[:, 0]
        rows[:len(e), 1] = e[:, 1]
        rows[:len(e), 2] = e[:, 2] | (e[:, 3] << 8)
        t.numpy()[:4 * n_pad] = rows.reshape(-1)

    def cap_install_edges(self, t, n_rows):
        rows = t.numpy()[:4 * n_rows].reshape(-1, 4).astype(np.int64)
        rows = rows[rows[:, 0] >= 0]
        self._edges = np.stack([rows[:, 0], rows[:, 1], rows[:, 2] & 0xff, rows[:, 2] >> 8], axis=1)
        self._fwd = np.bincount(rows[:, 0], minlength=self.n_reads)

    def _candidates(self, thr):
        """T: x joins when fwd(x) + #{y in T, y < x, (y, x) in E*} >= thr (rank order)."""
        back = np.zeros(self.n_reads, np.int64)
        adj = {}
        for a, b in self._edges[:, :2].tolist():
            adj.setdefault(a, []).append(b)
        T = []
        for x in range(self.n_reads):
            if self._fwd[x] + back[x] >= thr:
                T.append(x)
                for y in adj.get(x, ()):
                    back[y] += 1
        return T

    def _hit_lists(self, T, owned):
        """Per interval of each read of T (CSR order): the partner reads of its end-inclusive hits in
        the stand-in's search order (descending (start, -end, data position)), own read dropped."""
        c = self.csr
        chrom = np.asarray(c.iv_chrom)
        st, en = np.asarray(c.iv_start, np.int64), np.asarray(c.iv_end, np.int64)
        dp = np.asarray(c.data_pos, np.int64)
        off = np.asarray(c.read_off, np.int64)
        out = []
        for x in T:
            for k in range(off[x], off[x + 1]):
                if owned is not None and not owned[chrom[k]]:
                    out.append([])
                    continue
                h = np.flatnonzero((chrom == chrom[k]) & (st <= en[k]) & (en >= st[k]) & (self.read_of != x))
                order = sorted(h.tolist(), key=lambda p: (st[p], -en[p], dp[p]), reverse=True)
                out.append([int(self.read_of[p]) for p in order])
        return out

    def cap_local(self, edge_threshold=10):
        self._cap_thr = edge_threshold
        self._T = self._candidates(edge_threshold)
        lists = self._hit_lists(self._T, self.owned)
        self._cap_counts = np.array([len(x) for x in lists], np.int32)
        self._cap_hits = np.array([y for x in lists for y in x], np.int32)
        return int(self._cap_counts.size), int(self._cap_hits.size)

    def cap_copy_local(self, counts, hits):
        counts.numpy()[:self._cap_counts.size] = self._cap_counts
        hits.numpy()[:self._cap_hits.size] = self._cap_hits

    def cap_replay(self, counts, hits, pad, world):
        """Assemble the ranks' lists (each rank: its intervals' segments in interval order) and check
        them against the lists of an unfiltered index; then the capped graph is the oracle's loop."""
        nti = self._cap_counts.size
        cnt = counts.numpy()[:world * nti].reshape(world, nti)
        assert ((cnt > 0).sum(axis=0) <= 1).all(), 'an interval listed by two ranks'
        hv = hits.numpy()[:world * pad].reshape(world, pad)
        pos = [0] * world
        got = []
        for ti in range(nti):
            seg = []
            for w in range(world):
                m = int(cnt[w, ti])
                seg += hv[w, pos[w]:pos[w] + m].tolist()
                pos[w] += m
            got.append(seg)
        assert got == self._hit_lists(self._T, None)
        return self.apply_edge_cap(self._cap_thr)

    def apply_edge_cap(self, edge_threshold=10):
        from oracle import oracle as O
        c = self.csr
        cnt = np.diff(c.read_off)
        oc = O.OracleCSR(c.read_off, c.iv_chrom, c.iv_start, c.iv_end, c.iv_aln, np.repeat(c.read_qlen2, cnt),
                         np.repeat(c.read_nal, cnt), c.data_pos)
        qd, nd, ov = self.diffs
        o = O.run_core(oc, overlap=ov, use_cap=True, qlen_diff=qd, n_aln_diff=nd, edge_threshold=edge_threshold)
        self._edges = np.stack([o['edge_a'], o['edge_b'], o['edge_I'], o['edge_U']], axis=1).astype(np.int64)
        self._fwd = np.asarray(o['fwd'], np.int64)
        self._st = {'n_edges': len(self._edges), 'edge_capacity': self.edge_capacity,
                    'max_fwd': int(self._fwd.max()) if self._fwd.size else 0}
        return {'applied': 1}
