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
        self.prange = None                                 # the position split's (lo, hi, end)
        self._pset = None
        self.n_intervals = int(off[-1])
        # each interval's position in the (chrom, start)-sorted index: chromosome, then data order
        self.pos = np.empty(self.n_intervals, np.int64)
        self.pos[np.lexsort((np.asarray(csr.data_pos, np.int64), np.asarray(csr.iv_chrom, np.int64)))] = \
            np.arange(self.n_intervals)
        self.edge_capacity = 1 << 30
        self._edges = np.zeros((0, 4), np.int64)
        self._parent = np.arange(self.n_reads)
        self._st = {}

    # -- filter / index ------------------------------------------------------------------------
    def set_chrom_filter(self, owned):
        self.owned = None if owned is None else np.asarray(owned, dtype=bool)
        self.prange = None

    def _n_fwd(self):
        """Per sorted position q: #{p > q of its chromosome : start_p <= end_q} (end-inclusive hits)."""
        c = self.csr
        order = np.argsort(self.pos)
        ch = np.asarray(c.iv_chrom, np.int64)[order]
        st = np.asarray(c.iv_start, np.int64)[order]
        en = np.asarray(c.iv_end, np.int64)[order]
        nf = np.zeros(order.size, np.int64)
        for x in np.unique(ch):
            k = np.flatnonzero(ch == x)
            nf[k] = np.searchsorted(st[k], en[k], side='right') - np.arange(k.size) - 1
        return nf

    def has_data_order(self):
        return True

    def position_costs(self):
        nf = self._n_fwd()
        nt = (nf.size + 63) // 64
        tests = np.array([nf[64 * t:64 * t + 64].sum() for t in range(nt)], np.int64)
        reach = np.array([(np.arange(64 * t, min(nf.size, 64 * t + 64)) + nf[64 * t:64 * t + 64] + 1).max()
                          for t in range(nt)], np.int64)
        return tests, reach

    def set_position_filter(self, lo, hi, end):
        nf = self._n_fwd()
        q = np.arange(nf.size)
        sel = (q >= lo) & (q < hi)
        assert (q[sel] + nf[sel] < end).all(), 'the position range does not hold its forward windows'
        self.owned = None
        self.prange = self._pset = (int(lo), int(hi), int(end))

    def use_position_filter(self):
        assert self._pset is not None
        self.owned = None
        self.prange = self._pset

    def build_index(self):
        pass

    def reserve_edges(self, cap):
        pass

    # -- partition ------------------------------------------------------------------------------
    def _gate(self, a, b, qcut, ncut):
        """(passes, raises ZeroDivisionError) of the length gate (cluster.py:178-183)."""
        q1, q2 = int(self.csr.read_qlen2[a]), int(self.csr.read_qlen2[b])
        mn, mx = min(q1, q2), max(q1, q2)
        if mx == 0:
            return False, True
        if mn / mx >= qcut:
            return True, False
        n1, n2 = int(self.csr.read_nal[a]), int(self.csr.read_nal[b])
        mn, mx = min(n1, n2), max(n1, n2)
        if mx == 0:
            return False, True
        return mn / mx >= ncut, False

    def _entries(self, qcut, ncut, tiles=None):
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
            ra, rb = self.read_of[ks][:, None], self.read_of[ks][None, :]
            hit = (o >= 0) & (ra < rb)              # end-inclusive overlap of two different reads (:201)
            ok = hit & (o >= self.thr[ks][:, None]) & (o >= self.thr[ks][None, :])
            if self.prange is not None:             # the position split: the pair's lower position in [lo, hi)
                lower = np.minimum(self.pos[ks][:, None], self.pos[ks][None, :])
                inr = (lower >= self.prange[0]) & (lower < self.prange[1])
                hit &= inr
            x, y = np.nonzero(hit)
            for p, q, m in zip(ks[x].tolist(), ks[y].tolist(), ok[x, y].tolist()):
                a, b = int(self.read_of[p]), int(self.read_of[q])
                passes, zd = self._gate(a, b, qcut, ncut)
                if zd:
                    self._zd.add((a, b))            # listed, not raised (the edge cap decides)
                elif passes and m:
                    out.append((a << 39) | (b << 14) | (int(self.slot[p]) << 7) | int(self.slot[q]))
                    if tiles is not None:
                        tiles[min(int(self.pos[p]), int(self.pos[q])) // 64] += 1
        return np.array(out, dtype=np.int64)

    def position_entries(self, qlen_cut, nal_cut, pass_table, edge_threshold=10):
        """fslr_position_entries: match entries per 64-position tile of the full index."""
        tiles = np.zeros((self.pos.size + 63) // 64, np.int64)
        owned, prange, zd = self.owned, self.prange, getattr(self, '_zd', set())
        self.owned = self.prange = None
        try:
            self._zd = set()
            self._entries(qlen_cut, nal_cut, tiles)
        finally:
            self.owned, self.prange, self._zd = owned, prange, zd
        return tiles

    def sweep_partition(self, qlen_cut, nal_cut, pass_table, n_dest, block_shift, dst, edge_threshold=10):
        self._zd = set()
        ent = self._entries(qlen_cut, nal_cut)
        dest = (ent >> (39 + block_shift)) % n_dest
        order = np.argsort(dest, kind='stable')
        counts = np.bincount(dest, minlength=n_dest).astype(np.int64)
        if counts.sum() > dst.numel():
            return False, counts
        dst.numpy()[:ent.size] = ent[order]
        self._st = {'match_entries': int(ent.size), 'zd_pairs': len(self._zd)}
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
                    'max_fwd': int(fwd.max()) if fwd.size else 0, 'zd_pairs': len(getattr(self, '_zd', ()))}

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

    def local_forest(self, count=True):
        self.components()
        lab = self.labels().astype(np.int64)
        x = np.flatnonzero(lab != np.arange(self.n_reads))
        self._forest = np.stack([x, lab[x]], axis=1)
        return int(x.size) if count else None

    def forest_pairs_into(self, t, n_pad):
        pairs = np.full((n_pad, 2), -1, dtype=np.int32)
        pairs[:len(self._forest)] = self._forest
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

    def _candidates(self, thr, edges=None, fwd=None):
        """T: x joins when fwd(x) + #{y in T, y < x, (y, x) in E*} >= thr (rank order)."""
        edges = self._edges[:, :2] if edges is None else edges
        fwd = self._fwd if fwd is None else fwd
        back = np.zeros(self.n_reads, np.int64)
        adj = {}
        for a, b in edges.tolist():
            adj.setdefault(a, []).append(b)
        T = []
        for x in range(self.n_reads):
            if fwd[x] + back[x] >= thr:
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
        if getattr(self, '_gmode', False):
            g = self._g[self._g[:, 0] >= 0]
            self._T = self._candidates(edge_threshold, g, self._gfwd)
        else:
            self._T = self._candidates(edge_threshold)
        inT = set(self._T)
        if any(a not in inT or b not in inT for a, b in getattr(self, '_zd', ())):
            # a listed pair with a read outside T: that read's loop never breaks and visits it
            raise ZeroDivisionError('division by zero')
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

    # -- the sharded edge cap (fslr_cap_install_pairs ... fslr_cap_apply_changes) ------------------
    def sort_edges(self):
        if len(self._edges):
            self._edges = self._edges[np.lexsort((self._edges[:, 1], self._edges[:, 0]))]

    def cap_bwd_counts(self, edge_threshold, t):
        import torch
        e = self._edges
        self._r_thr = int(edge_threshold)
        self._rfwd = np.bincount(e[:, 0], minlength=self.n_reads) if len(e) else np.zeros(self.n_reads, np.int64)
        b = np.bincount(e[:, 1], minlength=self.n_reads) if len(e) else np.zeros(self.n_reads, np.int64)
        if t.dtype == torch.uint8:
            b = np.minimum(b, edge_threshold)
        t.numpy()[:self.n_reads] = b

    def cap_restrict(self, t):
        bwd = t.numpy()[:self.n_reads].astype(np.int64)
        e = self._edges
        keep = (self._rfwd[e[:, 0]] + bwd[e[:, 0]] >= self._r_thr) if len(e) else np.zeros(0, bool)
        rm = np.flatnonzero(keep)
        self._rmap = rm[np.argsort(e[rm, 0], kind='stable')]      # by lower read (one run per read)
        return int(self._rmap.size)

    def cap_copy_restricted(self, t, n_pad):
        pairs = np.full((n_pad, 2), -1, dtype=np.int32)
        pairs[:self._rmap.size] = self._edges[self._rmap, :2]
        t.numpy()[:n_pad] = pairs.view(np.int64)[:, 0]

    def cap_install_restricted(self, t, n_rows, world, rank):
        self.cap_install_pairs(t, n_rows, world, rank)
        self._restricted = True

    def cap_install_pairs(self, t, n_rows, world, rank):
        self._restricted = False
        self._g = t.numpy()[:n_rows].view(np.int32).reshape(-1, 2).astype(np.int64)
        self._gw, self._gr, self._gm = int(world), int(rank), int(n_rows) // int(world)
        v = self._g[:, 0] >= 0
        self._gfwd = np.bincount(self._g[v, 0], minlength=self.n_reads)
        self._gmode = True

    def cap_sizes(self):
        return len(self._T), int(self._cap_counts.size), int(self._cap_hits.size)

    def _ti_read(self):
        off = np.asarray(self.csr.read_off, np.int64)
        return np.repeat(np.arange(len(self._T)), [off[x + 1] - off[x] for x in self._T]).astype(np.int64)

    def cap_dep_local(self, t):
        """Roots (smallest t) of the forest of T-T hits on this rank's chromosomes; local hits per t."""
        nt = len(self._T)
        t_of = {x: k for k, x in enumerate(self._T)}
        par = list(range(nt))

        def find(x):
            while par[x] != x:
                x = par[x]
            return x
        tread = self._ti_read()
        hits = np.zeros(nt, np.int64)
        pos = 0
        for ti, cnt in enumerate(self._cap_counts.tolist()):
            tx = int(tread[ti])
            hits[tx] += cnt
            for y in self._cap_hits[pos:pos + cnt].tolist():
                if y in t_of:
                    a, b = find(tx), find(t_of[y])
                    if a != b:
                        par[max(a, b)] = min(a, b)
            pos += cnt
        out = t.numpy()
        out[:nt] = [find(k) for k in range(nt)]
        out[nt:2 * nt] = hits

    def cap_shard_plan(self, gathered, world, rank):
        nt = len(self._T)
        g = gathered.numpy()[:world * 2 * nt].reshape(world, 2 * nt).astype(np.int64)
        par = list(range(nt))

        def find(x):
            while par[x] != x:
                x = par[x]
            return x
        for w in range(world):
            for k in range(nt):
                a, b = find(k), find(int(g[w, k]))
                if a != b:
                    par[max(a, b)] = min(a, b)
        comp = np.array([find(k) for k in range(nt)], np.int64)
        cost = g[:, nt:].sum(axis=0) + 1
        ccost = np.bincount(comp, weights=cost, minlength=nt).astype(np.int64)
        roots = sorted(set(comp.tolist()), key=lambda r: (-ccost[r], r))
        load = np.zeros(world, np.int64)
        droot = {}
        for k, r in enumerate(roots):
            if k < 256:                  # the largest onto the least-loaded rank (k_cap_assign_head)
                d = int(np.argmin(load))
                load[d] += ccost[r]
            else:                        # the rest dealt in snake order (k_cap_assign_tail)
                j = k - 256
                d = world - 1 - j % world if (j // world) & 1 else j % world
            droot[r] = d
        self._comp = comp
        self._tdest = np.array([droot[c] for c in comp.tolist()], np.int64)
        tread = self._ti_read()
        dti = self._tdest[tread]
        self._tsorted = np.argsort(dti, kind='stable')
        ti_d = np.bincount(dti, minlength=world).astype(np.int64)
        hits_d = np.bincount(dti, weights=self._cap_counts, minlength=world).astype(np.int64)
        self._mine = self._tsorted[ti_d[:rank].sum():ti_d[:rank + 1].sum()]
        return ti_d, hits_d

    def cap_shard_pack(self, counts, hits):
        off = np.concatenate([[0], np.cumsum(self._cap_counts)])
        c = self._cap_counts[self._tsorted]
        counts.numpy()[:c.size] = c
        h = [self._cap_hits[off[ti]:off[ti + 1]] for ti in self._tsorted.tolist()]
        if h:
            h = np.concatenate(h)
            hits.numpy()[:h.size] = h

    def cap_replay_shard(self, counts, hits):
        """Assemble this rank's T-intervals' lists from the received ones and check them against an
        unfiltered index's; the changes of the rows it decides come from the oracle's capped graph."""
        W, nm = self._gw, self._mine.size
        rc = counts.numpy()[:W * nm].reshape(W, nm)
        assert ((rc > 0).sum(axis=0) <= 1).all(), 'an interval listed by two ranks'
        rh = hits.numpy()
        pos = np.concatenate([[0], np.cumsum(rc.reshape(-1))])
        full = self._hit_lists(self._T, None)
        for i, ti in enumerate(self._mine.tolist()):
            seg = []
            for w in range(W):
                k = w * nm + i
                seg += rh[pos[k]:pos[k + 1]].tolist()
            assert seg == full[ti]
        from oracle import oracle as O
        c = self.csr
        cnt = np.diff(c.read_off)
        oc = O.OracleCSR(c.read_off, c.iv_chrom, c.iv_start, c.iv_end, c.iv_aln, np.repeat(c.read_qlen2, cnt),
                         np.repeat(c.read_nal, cnt), c.data_pos)
        qd, nd, ov = self.diffs
        o = O.run_core(oc, overlap=ov, use_cap=True, qlen_diff=qd, n_aln_diff=nd, edge_threshold=self._cap_thr)
        kept = set(zip(np.asarray(o['edge_a']).tolist(), np.asarray(o['edge_b']).tolist()))
        t_of = {x: k for k, x in enumerate(self._T)}
        chg = []
        for k, (a, b) in enumerate(self._g.tolist()):
            if a < 0:
                continue
            t = t_of.get(a, t_of.get(b, -1))
            if t < 0 or self._tdest[t] != self._gr:
                continue
            w = 0 if (a, b) in kept else (1 if (b, a) in kept else 2)
            if w:
                chg.append((k << 2) | w)
        self._chg = np.array(chg, np.int32)
        return len(chg), {'applied': 1, 'candidates': len(self._T), 'capped': 0,
                          'hits': int(sum(len(full[ti]) for ti in self._mine.tolist())), 'pairs': 0}

    def cap_copy_changes(self, t, n_pad):
        out = np.full(n_pad, -1, np.int32)
        out[:self._chg.size] = self._chg
        t.numpy()[:n_pad] = out

    def cap_apply_changes(self, t, n):
        ch = t.numpy()[:n].astype(np.int64)
        ch = ch[ch >= 0]
        who = np.zeros(len(self._g), np.int64)
        who[ch >> 2] = ch & 3
        m, r = self._gm, self._gr
        loc = self._edges
        if self._restricted:                     # this rank's block of S rows back onto its edges
            wl = np.zeros(len(loc), np.int64)
            wl[self._rmap] = who[r * m:r * m + self._rmap.size]
            lf = self._rfwd
        else:
            wl = who[r * m:r * m + len(loc)]
        keep = wl != 2
        e = loc[keep].copy()
        fl = wl[keep] == 1
        e[fl, 0], e[fl, 1] = loc[keep][fl, 1], loc[keep][fl, 0]
        self._edges = e
        self._fwd = np.bincount(e[:, 0], minlength=self.n_reads) if len(e) else np.zeros(self.n_reads, np.int64)
        formed = self._gfwd.copy()
        for k in np.flatnonzero(who).tolist():
            a, b = self._g[k]
            formed[a] -= 1
            if who[k] == 1:
                formed[b] += 1
        if self._restricted:                     # reads with no gathered row: their own edges
            formed += np.where(self._gfwd == 0, lf, 0)
        self._gmode = False
        self._st = {'n_edges': len(e), 'edge_capacity': self.edge_capacity, 'max_fwd': int(formed.max())}
        return {'applied': 1, 'max_fwd': int(formed.max()), 'candidates': len(self._T), 'capped': 0, 'hits': 0,
                'pairs': 0, 'dropped': int((who == 2).sum()), 'backward': int((who == 1).sum())}
