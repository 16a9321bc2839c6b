#!/usr/bin/env python3
"""Host stages of `fslr --skip-alignment` without a GPU: the CLI's clustering block on a
`.mappings.bed` (DIR/x.mappings.bed + DIR/x.bwa_dodi.bam) with the device query replaced by a
stand-in graph (reads in groups of three), so the read / prepare / CSR / write stages are timed as
the CLI runs them.  Prints the CLI's `timings_s` line; --profile adds the top cProfile entries.

    python tools/cli_stages_cpu.py DIR [--pandas-io] [--profile]
"""
import cProfile
import io
import os
import pstats
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from fslr_amd import cluster  # noqa: E402


def stand_in(trees, data, overlap, cuts, thr, qlen_diff, diff):
    csr = data.csr()
    n = csr.n_reads
    a = np.arange(n, dtype=np.int32)
    keep = a % 3 != 0
    lab = (a // 3 * 3).astype(np.int32)
    z = np.zeros(int(keep.sum()), np.int32)
    return cluster.RawGraph(data, csr, lab, a[keep] - 1, a[keep], z + 1, z + 2, np.zeros(n, np.int32),
                            {'engine': 'stand-in'})


def main():
    d = sys.argv[1]
    cluster.build_interval_trees = lambda data, device=None, n_gpus=1, ctx=None: None
    cluster._open_context = lambda device=None: None
    cluster.query_graph = stand_in
    from click.testing import CliRunner
    from fslr_amd.main import pipeline
    io_flag = '--pandas-io' if '--pandas-io' in sys.argv else '--native-io'
    args = ['--name', 'x', '--out', d, '--ref', 'unused.fa', '--primers', '21q1', '--skip-alignment', '--timings',
            io_flag]
    pr = cProfile.Profile() if '--profile' in sys.argv else None
    if pr:
        pr.enable()
    res = CliRunner().invoke(pipeline, args, catch_exceptions=False)
    if pr:
        pr.disable()
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats('tottime').print_stats(30)
        print(s.getvalue())
    print(res.output)


if __name__ == '__main__':
    main()
