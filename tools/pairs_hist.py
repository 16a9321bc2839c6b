"""Group sizes of k_sweep_pairs at cfg3, or cfg5 with --cfg5 (measurement build: tools/build_variant.sh hist
-DFSLR_PAIRS_HIST).
Usage (GPU box): FSLR_LIB=fslr_amd/libfslr_hip_hist.so FSLR_ALLOW_STALE=1 python tools/pairs_hist.py OUT.json [--cfg5]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from fslr_amd import _lib, synth  # noqa: E402
from fslr_amd.prep import fold_overlap_threshold, pass_table  # noqa: E402


def main():
    cfg5 = '--cfg5' in sys.argv
    s = synth.generate(10_000_000, 64, 13, dist='zipf') if cfg5 else synth.generate(1_000_000, 16, 11)
    csr = s.interval_data().csr()
    del s
    ctx = _lib.Context(0)
    ctx.load_csr(csr, fold_overlap_threshold(csr.iv_aln, 0.8))
    ctx.reserve_edges(3 * csr.n_reads if cfg5 else 12 * csr.n_reads)
    ctx.build_index()
    st = ctx.run_query(0.96, 0.75, pass_table([1, 1, 0.66, 0.66, 0.66, 0.5]), 10, engine='sweep')
    c = ctx.counters(80).astype(np.int64)
    bins = c[48:64]
    groups = int(bins.sum())
    out = {'input': 'cfg5: 10M reads x 1-64 zipf, seed 13' if cfg5 else 'cfg3: 1M reads x 1-16, seed 11',
           'match_entries': int(st['match_entries']),
           'groups': groups, 'long_runs': int(c[42]), 'read_pairs_in_groups': int(c[43]),
           'runs_in_groups': int(c[44]), 'long_run_entries': int(c[45]), 'long_run_pass_steps': int(c[46]),
           'longest_run': int(c[47]), 'bucketed_runs': int(c[40]), 'bucketed_run_entries': int(c[41]),
           'group_size_hist': {f'{8 * k + 1}-{8 * k + 8}': int(v) for k, v in enumerate(bins)},
           'mean_group_entries': None}
    out['share_le_64'] = float(bins[:8].sum() / max(1, groups))
    ent = sum((8 * k + 4.5) * int(v) for k, v in enumerate(bins))
    out['mean_group_entries'] = ent / max(1, groups)
    # wave-clock sums per phase of k_sweep_pairs (s_memtime: its reads wait for the wave's LDS ops)
    ph = c[68:74].astype(np.float64)
    names = ['window_heads', 'sort', 'segment_setup', 'segment_eval', 'tail', 'long_runs']
    out['phase_clock_share'] = {k: float(v / max(1.0, ph.sum())) for k, v in zip(names, ph)}
    print(json.dumps(out, indent=1))
    with open(sys.argv[1], 'w') as fh:
        json.dump(out, fh, indent=1)
    ctx.close()


if __name__ == '__main__':
    main()
