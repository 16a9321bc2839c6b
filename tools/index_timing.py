#!/usr/bin/env python3
"""Device time of build_index alone (median over --steps), for index-build variants.

    FSLR_LIB=fslr_amd/libfslr_hip_<variant>.so python tools/index_timing.py [--reads 1000000]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--reads', type=int, default=1_000_000)
    ap.add_argument('--lmax', type=int, default=16)
    ap.add_argument('--seed', type=int, default=11)
    ap.add_argument('--steps', type=int, default=20)
    args = ap.parse_args()
    import torch
    from fslr_amd import _lib, synth
    from fslr_amd.prep import fold_overlap_threshold
    csr = synth.generate(args.reads, args.lmax, args.seed).interval_data().csr()
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    ctx = _lib.Context(0, stream=stream.cuda_stream)
    ctx.load_csr(csr, fold_overlap_threshold(csr.iv_aln, 0.8))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t = []
    for k in range(args.steps + 2):
        e0.record(stream)
        ctx.build_index()
        e1.record(stream)
        torch.cuda.synchronize()
        if k >= 2:
            t.append(e0.elapsed_time(e1))
    print(json.dumps({'lib': os.environ.get('FSLR_LIB', 'default'), 'index_ms_median': float(np.median(t)),
                      'index_ms_min': float(np.min(t))}), flush=True)
    ctx.close()


if __name__ == '__main__':
    main()
