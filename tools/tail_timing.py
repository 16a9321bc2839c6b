#!/usr/bin/env python3
"""Per-read timing of the pair kernel per query shard (FSLR_SECTION_PROF build).

    python tools/tail_timing.py [--worlds 1,8]

For shard 0 of each W: wave-time spread (mean / min / max) and the per-read
cycles (s_memtime) of query_kernel, binned by start time inside the wave, by
the read's interval count L and by rank decile.
"""
import argparse
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
os.environ.setdefault('FSLR_LIB', os.path.join(REPO, 'fslr_amd', 'libfslr_hip_prof.so'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--reads', type=int, default=1_000_000)
    ap.add_argument('--lmax', type=int, default=16)
    ap.add_argument('--seed', type=int, default=11)
    ap.add_argument('--dist', default='uniform')
    ap.add_argument('--worlds', default='1,8')
    ap.add_argument('--save', default='', help='prefix: save raw per-read diagnostics as npz')
    args = ap.parse_args()
    import numpy as np
    from fslr_amd import _lib, synth
    from fslr_amd.prep import fold_overlap_threshold, pass_table
    csr = synth.generate(args.reads, args.lmax, args.seed, dist=args.dist).interval_data().csr()
    n = csr.n_reads
    L = np.diff(csr.read_off)
    ctx = _lib.Context(0)
    ctx.load_csr(csr, fold_overlap_threshold(csr.iv_aln, 0.8))
    ctx.reserve_edges(12 * n)
    pt = pass_table([1, 1, 0.66, 0.66, 0.66, 0.5])
    lib = _lib.load()
    lib.fslr_prof_read_diag.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    out = {}
    for W in [int(x) for x in args.worlds.split(',')]:
        ctx.set_shard(0, W)
        for _ in range(2):
            ctx.build_index()
            ctx.query_shard(1 - 0.04, 1 - 0.25, pt, 0, W)
            ctx.sync()
        c = ctx.counters(80).astype(np.float64)
        d = np.zeros(2 * n, np.uint64)
        assert lib.fslr_prof_read_diag(ctx._h, d.ctypes.data) == 0
        own = ((np.arange(n) >> 6) % W) == 0
        rt = d[0::2][own].astype(np.float64)            # s_memrealtime (100 MHz) at read start
        w1 = d[1::2][own]
        dt = (w1 & np.uint64(0xffffffff)).astype(np.float64)
        smid = ((w1 >> np.uint64(32)) & np.uint64(0xffff)).astype(np.int64)
        it = (w1 >> np.uint64(48)).astype(np.int64)
        Lo = L[own]
        nw = c[60]
        t0 = rt - rt.min()
        tb = np.linspace(0, t0.max() + 1, 17)
        bt = np.clip(np.searchsorted(tb, t0, side='right') - 1, 0, 15)
        by_time = [[round(float(tb[i]) / 100.0, 1), int((bt == i).sum()),
                    round(float(dt[bt == i].mean())) if (bt == i).any() else 0] for i in range(16)]   # us
        by_L = [[int(l), int((Lo == l).sum()), round(float(dt[Lo == l].mean()))] for l in np.unique(Lo)]
        rk = np.flatnonzero(own)
        dec = np.minimum(rk * 10 // n, 9)
        by_rank = [[int(i), round(float(dt[dec == i].mean()))] for i in range(10) if (dec == i).any()]
        by_iter = [[int(k), int((it == k).sum()), round(float(dt[it == k].mean())),
                    round(float(t0[it == k].mean()) / 100.0, 1)] for k in np.unique(it)]
        xcc = smid >> 6
        by_xcc = [[int(x), int((xcc == x).sum()), round(float(dt[xcc == x].mean()))] for x in np.unique(xcc)]
        out[W] = {'waves': int(nw), 'mean_wave_cycles': c[55] / max(nw, 1), 'max_wave_cycles': c[58],
                  'min_wave_cycles': c[59], 'mean_read_cycles': float(dt.mean()),
                  'p99_read_cycles': float(np.percentile(dt, 99)), 'max_read_cycles': float(dt.max()),
                  'span_us': float(t0.max()) / 100.0, 'by_time_us': by_time, 'by_L': by_L,
                  'by_rank_decile': by_rank, 'by_iter': by_iter, 'by_xcc': by_xcc}
        print(W, json.dumps(out[W]), file=sys.stderr, flush=True)
        if args.save:
            np.savez_compressed(f'{args.save}_W{W}.npz', rank=rk, rt=d[0::2][own], w1=d[1::2][own], L=Lo)
    print(json.dumps(out))
    ctx.close()


if __name__ == '__main__':
    main()
