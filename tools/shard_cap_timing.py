#!/usr/bin/env python3
"""Per-rank phase timing of the chromosome-split step WITH the sharded edge-cap replay,
measured on ONE GPU with W contexts (one per rank, each indexing its own chromosomes).

Every phase runs rank after rank (a synchronize around each), so each rank's time is its own:
  part[r]   build_index (filtered) + fslr_sweep_partition
  eval[d]   fslr_sweep_evaluate of the entries destined to d + the copy of its edges for the gather
  cap_local[r]  fslr_cap_install_restricted (or _pairs) + fslr_cap_local + fslr_cap_dep_local (closure
                over the gathered rows, T's local hit lists, the local T-T forest)
  cap_plan[r]   fslr_cap_shard_plan + fslr_cap_shard_pack
  cap_replay[r] fslr_cap_replay_shard (this rank's components)
  cap_apply[r]  fslr_cap_apply_changes + fslr_local_forest (its capped edges' forest)
  cap_merge[r]  fslr_components_from_pairs over the gathered forests (the capped graph's labels)
  (the edge sort before the gather, fslr_sort_edges, and with the restricted gather (--gather, default)
  fslr_cap_bwd_counts + fslr_cap_restrict are reported as parts before cap_local; the counts' sum over
  ranks is priced as a ring all_reduce)
The exchanges cannot run on one GPU; they are priced from the bytes each rank moves at an assumed
per-GPU xGMI rate (--xgmi-gbs) plus a fixed latency per collective (--coll-us), as
tools/shard_timing.py does.  The single-context step (index + sweep query + fslr_apply_edge_cap +
components) is the W = 1 baseline; every rank's labels are checked against it.

    python tools/shard_cap_timing.py --reads 10000000 --lmax 64 --dist zipf --seed 13 --worlds 8
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--reads', type=int, default=10_000_000)
    ap.add_argument('--lmax', type=int, default=64)
    ap.add_argument('--dist', default='zipf')
    ap.add_argument('--seed', type=int, default=13)
    ap.add_argument('--worlds', default='8')
    ap.add_argument('--reps', type=int, default=3)
    ap.add_argument('--edge-threshold', type=int, default=10)
    ap.add_argument('--xgmi-gbs', type=float, default=300.0)
    ap.add_argument('--coll-us', type=float, default=30.0)
    ap.add_argument('--gather', choices=['restricted', 'full'], default='restricted',
                    help='gather the rows of S only (the default of dist.SweepShard) or every E* row')
    args = ap.parse_args()
    restricted = args.gather == 'restricted'
    import torch
    from fslr_amd import _lib, synth
    from fslr_amd.dist import chrom_counts_of, chrom_owner
    from fslr_amd.prep import fold_overlap_threshold, pass_table

    t = time.perf_counter()
    s = synth.generate(args.reads, args.lmax, args.seed, dist=args.dist)
    csr = s.interval_data().csr()
    del s
    log(f'data: {csr.n_reads} reads, {csr.n_intervals} intervals in {time.perf_counter() - t:.0f}s')
    n = csr.n_reads
    thr = fold_overlap_threshold(csr.iv_aln, 0.8)
    pt = pass_table([1, 1, 0.66, 0.66, 0.66, 0.5])
    qc, nc, et = 1 - 0.04, 1 - 0.25, args.edge_threshold
    dev = torch.device('cuda', 0)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    gbs, cl = args.xgmi_gbs * 1e6, args.coll_us / 1000     # bytes per ms, ms

    def sync():
        torch.cuda.synchronize()

    def timed_once(fn):
        sync()
        t0 = time.perf_counter()
        r = fn()
        sync()
        return 1000 * (time.perf_counter() - t0), r

    # W = 1: the single-context step with the cap replay
    c1 = _lib.Context(0, stream=stream.cuda_stream)
    c1.load_csr(csr, thr)
    c1.reserve_edges(12 * n)
    one = []
    for rep in range(args.reps + 1):
        sync()
        t0 = time.perf_counter()
        c1.build_index()
        c1.query(qc, nc, pt, et, engine='sweep')
        t1 = time.perf_counter()
        c1.sync()
        t1 = time.perf_counter()
        cap1 = c1.apply_edge_cap(et)
        t2 = time.perf_counter()
        c1.components()
        sync()
        t3 = time.perf_counter()
        if rep:
            one.append((1000 * (t1 - t0), 1000 * (t2 - t1), 1000 * (t3 - t0)))
    one = np.median(np.array(one), axis=0)
    ref_labels = c1.labels()
    st1 = c1.stats()
    log(f'W=1: query {one[0]:.3f} ms, cap {one[1]:.3f} ms, step {one[2]:.3f} ms; cap {cap1}')
    c1.close()
    out = {'gather': args.gather, 'workload': f'{n} reads x 1-{args.lmax} ({args.dist}), seed {args.seed}', 'n_reads': n,
           'n_intervals': int(csr.n_intervals), 'single': {'query_ms': one[0], 'cap_ms': one[1], 'step_ms': one[2],
                                                           'cap': cap1, 'edges': int(st1['n_edges'])},
           'xgmi_gbs_assumed': args.xgmi_gbs, 'collective_latency_us': args.coll_us, 'worlds': []}
    counts = chrom_counts_of(csr)
    for W in [int(x) for x in args.worlds.split(',')]:
        owner = chrom_owner(counts, W)
        ctx = []
        for r in range(W):
            c = _lib.Context(0, stream=stream.cuda_stream)
            c.load_csr(csr, thr)
            c.reserve_edges(max(1 << 16, int(2.5 * st1['n_edges'] / W) + 4096))
            c.set_chrom_filter(owner == r if W > 1 else None)
            ctx.append(c)
        ph = {k: [[] for _ in range(W)] for k in ('part', 'eval', 'cap_local', 'cap_plan', 'cap_replay', 'cap_apply',
                                                     'cap_merge')}
        model = []
        sub = {}
        for rep in range(args.reps + 1):
            segs, sent = [[] for _ in range(W)], []
            for r in range(W):
                buf = torch.empty(max(1 << 16, int(1.3 * st1['match_entries'] / W) + 4096) if 'match_entries' in st1
                                  else 1 << 24, dtype=torch.int64, device=dev)

                def p():
                    ctx[r].build_index()
                    return ctx[r].sweep_partition(qc, nc, pt, W, 6, buf, et)
                ms, (ok, cnt) = timed_once(p)
                if not ok:
                    buf = torch.empty(int(cnt.sum() * 1.1) + 4096, dtype=torch.int64, device=dev)
                    ms, (ok, cnt) = timed_once(p)
                ph['part'][r].append(ms)
                pos = np.concatenate([[0], np.cumsum(cnt)])
                for d in range(W):
                    segs[d].append(buf[pos[d]:pos[d + 1]].clone())
                sent.append(cnt)
                del buf
            ne = []
            for d in range(W):
                ent = torch.cat(segs[d])
                segs[d] = None
                ms, _ = timed_once(lambda: ctx[d].sweep_evaluate(qc, nc, pt, ent, ent.numel(), et))
                ne.append(ctx[d].stats()['n_edges'])
                ph['eval'][d].append(ms)
                del ent
            for d in range(W):
                # (the restricted gather sorts only its rows, inside fslr_cap_restrict)
                ms, _ = timed_once(lambda: None if restricted else ctx[d].sort_edges())
                sub.setdefault('sort', [[] for _ in range(W)])[d].append(ms)
            bwd_ms = 0.0
            if restricted:
                # the rows of S only: backward counts per rank, summed (all_reduce), then each rank's rows
                dt = torch.uint8 if W * et <= 255 else torch.int32
                bl = [torch.empty(n, dtype=dt, device=dev) for _ in range(W)]
                for d in range(W):
                    ms, _ = timed_once(lambda: ctx[d].cap_bwd_counts(et, bl[d]))
                    sub.setdefault('bwd_counts', [[] for _ in range(W)])[d].append(ms)
                bsum = torch.stack([b.to(torch.int32) for b in bl]).sum(dim=0).to(dt)
                del bl
                nrs = []
                for d in range(W):
                    ms, nr = timed_once(lambda: ctx[d].cap_restrict(bsum))
                    sub.setdefault('restrict', [[] for _ in range(W)])[d].append(ms)
                    nrs.append(nr)
                del bsum
                esz = 1 if dt == torch.uint8 else 4
                bwd_ms = 0.0 if W == 1 else 2 * (W - 1) / W * n * esz / gbs + 2 * cl   # + the counts' all_reduce
                m = max(1, max(nrs))
                rows = torch.empty(W * m, dtype=torch.int64, device=dev)
                for d in range(W):
                    ctx[d].cap_copy_restricted(rows[d * m:(d + 1) * m], m)
                if rep == 0:
                    out.setdefault('restrict', {})[W] = {'rows': int(sum(ne)), 'rows_in_S': int(sum(nrs))}
                    log('restricted gather:', out['restrict'][W])
            else:
                m = max(1, max(ne))
                rows = torch.empty(W * m, dtype=torch.int64, device=dev)
                for d in range(W):
                    ctx[d].edges_into(rows[d * m:(d + 1) * m], m)
            if rep == 0 and W > 1 and not restricted:
                # diagnostics: the rows whose lower read can join the candidates (total E* degree >= the cap)
                rw = rows.cpu().numpy().view(np.int32).reshape(-1, 2)
                rw = rw[rw[:, 0] >= 0]
                deg = np.bincount(rw[:, 0], minlength=n) + np.bincount(rw[:, 1], minlength=n)
                S = deg >= et
                out.setdefault('restrict', {})[W] = {'rows': int(rw.shape[0]), 'S': int(S.sum()),
                                                     'rows_lower_in_S': int(S[rw[:, 0]].sum())}
                log('restricted gather:', out['restrict'][W])
                del rw, deg, S
            nts = []
            tinfo = []
            for r in range(W):
                m1, _ = timed_once(lambda: (ctx[r].cap_install_restricted if restricted else ctx[r].cap_install_pairs)(
                    rows, W * m, W, r))
                m2, _ = timed_once(lambda: ctx[r].cap_local(et))
                nt = ctx[r].cap_sizes()[0]
                ti = torch.empty(max(1, 2 * nt), dtype=torch.int32, device=dev)
                m3, _ = timed_once(lambda: ctx[r].cap_dep_local(ti))
                ph['cap_local'][r].append(m1 + m2 + m3)
                sub.setdefault('install', [[] for _ in range(W)])[r].append(m1)
                sub.setdefault('closure_hits', [[] for _ in range(W)])[r].append(m2)
                sub.setdefault('dep_local', [[] for _ in range(W)])[r].append(m3)
                nts.append(nt)
                tinfo.append(ti[:2 * nt])
            nt = nts[0]
            assert all(x == nt for x in nts)
            tg = torch.cat(tinfo) if nt else torch.zeros(1, dtype=torch.int32, device=dev)
            sends = []
            for r in range(W):
                def pl():
                    ti_d, hits_d = ctx[r].cap_shard_plan(tg, W, r)
                    cs = torch.empty(max(1, int(ti_d.sum())), dtype=torch.int32, device=dev)
                    hs = torch.empty(max(1, int(hits_d.sum())), dtype=torch.int32, device=dev)
                    ctx[r].cap_shard_pack(cs, hs)
                    return ti_d, hits_d, cs, hs
                ms, snd = timed_once(pl)
                ph['cap_plan'][r].append(ms)
                sends.append(snd)
            ti_all = sends[0][0]
            hits_mat = np.array([s_[1] for s_ in sends])        # [source, dest]
            chg_n, parts = [], []
            for r in range(W):
                nm = int(ti_all[r])
                rc = torch.cat([s_[2][int(ti_all[:r].sum()):int(ti_all[:r].sum()) + nm] for s_ in sends]) if nm \
                    else torch.zeros(1, dtype=torch.int32, device=dev)
                rh_parts = []
                for w_, s_ in enumerate(sends):
                    o = int(hits_mat[w_, :r].sum())
                    rh_parts.append(s_[3][o:o + int(hits_mat[w_, r])])
                rh = torch.cat(rh_parts) if hits_mat[:, r].sum() else torch.zeros(1, dtype=torch.int32, device=dev)
                ms, (nch, part) = timed_once(lambda: ctx[r].cap_replay_shard(rc, rh))
                ph['cap_replay'][r].append(ms)
                chg_n.append(nch)
                parts.append(part)
            pad = max(1, max(chg_n))
            cg = torch.empty(W * pad, dtype=torch.int32, device=dev)
            for r in range(W):
                ctx[r].cap_copy_changes(cg[r * pad:(r + 1) * pad], pad)
            caps, fps = [], []
            for r in range(W):
                ms, cp = timed_once(lambda: ctx[r].cap_apply_changes(cg, W * pad))
                m4, fp = timed_once(lambda: ctx[r].local_forest())
                ph['cap_apply'][r].append(ms + m4)
                caps.append(cp)
                fps.append(fp)
            mf = max(1, max(fps))
            fg = torch.empty(W * mf, dtype=torch.int64, device=dev)
            for r in range(W):
                ctx[r].forest_pairs_into(fg[r * mf:(r + 1) * mf], mf)
            for r in range(W):
                ms, _ = timed_once(lambda: ctx[r].components_from_pairs(fg, W * mf))
                ph['cap_merge'][r].append(ms)
            if rep == 0:
                for r in range(W):
                    assert np.array_equal(ctx[r].labels(), ref_labels), f'rank {r}: labels differ from one context'
                assert sum(c.stats()['n_edges'] for c in ctx) == st1['n_edges']
                assert caps[0]['dropped'] == cap1['dropped'] and caps[0]['backward'] == cap1['backward']
                assert sum(p_['capped'] for p_ in parts) == cap1['capped']
            sent = np.array(sent)
            off_rank = np.array([sent[r].sum() - sent[r, r] for r in range(W)])
            recv = sent.sum(axis=0)
            a2a = 0.0 if W == 1 else 8 * max(off_rank.max(), (recv - np.diag(sent)).max()) / gbs + 2 * cl
            gath = 0.0 if W == 1 else 8 * m * (W - 1) / gbs + cl
            tg_ms = 0.0 if W == 1 else 8 * nt * (W - 1) / gbs + cl
            cnt_ms = 0.0 if W == 1 else 4 * int(ti_all.max()) * (W - 1) / gbs + cl
            hoff = np.array([hits_mat[w_].sum() - hits_mat[w_, w_] for w_ in range(W)])
            hin = np.array([hits_mat[:, w_].sum() - hits_mat[w_, w_] for w_ in range(W)])
            hits_ms = 0.0 if W == 1 else 4 * max(hoff.max(), hin.max()) / gbs + 2 * cl
            chg_ms = 0.0 if W == 1 else 4 * pad * (W - 1) / gbs + 2 * cl     # + the counts' all_gather
            fgath_ms = 0.0 if W == 1 else 8 * mf * (W - 1) / gbs + 2 * cl    # + the count's all_reduce
            model.append({'a2a_ms': a2a, 'gather_ms': gath, 'bwd_allreduce_ms': bwd_ms, 'gather_rows_per_rank': m, 'tinfo_gather_ms': tg_ms, 'counts_a2a_ms': cnt_ms,
                          'hits_a2a_ms': hits_ms, 'changes_gather_ms': chg_ms, 'forest_gather_ms': fgath_ms,
                          'forest_pairs': fps, 'nt': nt, 'changes': chg_n,
                          'hits_to': hits_mat.sum(axis=0).tolist(), 'entries_sent': sent.sum(axis=1).tolist(),
                          'edges_per_rank': ne})
        med = {k: [float(np.median(v[r][1:])) for r in range(W)] for k, v in ph.items()}
        mdl = model[-1]
        smed = {k: [float(np.median(v[r][1:])) for r in range(W)] for k, v in sub.items()}
        pre = max(smed['sort'])
        if restricted:
            pre += max(smed['bwd_counts']) + mdl['bwd_allreduce_ms'] + max(smed['restrict'])
        cap_ms = (pre + max(med['cap_local']) + mdl['tinfo_gather_ms']
                  + max(med['cap_plan']) + mdl['counts_a2a_ms'] + mdl['hits_a2a_ms'] + max(med['cap_replay'])
                  + mdl['changes_gather_ms'] + max(med['cap_apply']) + mdl['forest_gather_ms'] + max(med['cap_merge']))
        step = (max(med['part']) + mdl['a2a_ms'] + max(med['eval']) + cl + mdl['gather_ms'] + cap_ms)
        log('cap_local parts (max over ranks):', {k: round(max(v), 3) for k, v in smed.items()})
        row = {'W': W, 'phase_ms_per_rank': med, 'cap_local_parts_ms': smed, 'model': mdl,
               'cap_ms_per_rank_projected': cap_ms,
               'projected_step_ms': step, 'projected_speedup': one[2] / step,
               'single_cap_ms': one[1], 'cap_speedup': one[1] / cap_ms}
        log(f'W={W}: part {max(med["part"]):.3f}, eval {max(med["eval"]):.3f}, cap local {max(med["cap_local"]):.3f} '
            f'plan {max(med["cap_plan"]):.3f} replay {max(med["cap_replay"]):.3f} apply {max(med["cap_apply"]):.3f} '
            f'merge {max(med["cap_merge"]):.3f} '
            f'ms; cap per rank {cap_ms:.3f} ms (one GPU {one[1]:.3f}); step {step:.3f} ms ({one[2] / step:.2f}x)')
        out['worlds'].append(row)
        print(json.dumps(row), flush=True)
        for c in ctx:
            c.close()
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
