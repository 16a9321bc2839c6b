"""Wave-clock split of k_sweep<2> at cfg3 (measurement build: tools/build_variant.sh sclock -DFSLR_SWEEP_CLOCK).
Usage (GPU box): FSLR_LIB=fslr_amd/libfslr_hip_sclock.so FSLR_ALLOW_STALE=1 python tools/sweep_clock.py OUT.json"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from fslr_amd import _lib, synth  # noqa: E402
from fslr_amd.prep import fold_overlap_threshold, pass_table  # noqa: E402


def main():
    s = synth.generate(1_000_000, 16, 11)
    csr = s.interval_data().csr()
    ctx = _lib.Context(0)
    ctx.load_csr(csr, fold_overlap_threshold(csr.iv_aln, 0.8))
    ctx.reserve_edges(12 * csr.n_reads)
    ctx.build_index()
    ctx.run_query(0.96, 0.75, pass_table([1, 1, 0.66, 0.66, 0.66, 0.5]), 10, engine='sweep')
    c = ctx.counters(80).astype(np.float64)
    ph = c[68:72]
    names = ['tail', 'item_map', 'steps', 'tile_header']
    out = {'input': 'cfg3: 1M reads x 1-16, seed 11', 'note': 's_memtime reads wait for the wave\'s LDS ops',
           'phase_clock_share': {k: float(v / max(1.0, ph.sum())) for k, v in zip(names, ph)}}
    print(json.dumps(out, indent=1))
    with open(sys.argv[1], 'w') as fh:
        json.dump(out, fh, indent=1)
    ctx.close()


if __name__ == '__main__':
    main()
