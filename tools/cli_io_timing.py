"""End-to-end `fslr --skip-alignment` wall time with the native reader/writer vs pandas I/O.

Usage: python tools/cli_io_timing.py N_READS LMAX SEED OUT_JSON [DIST] [FLAGS]
  DIST: uniform (default) or zipf; FLAGS: comma-separated I/O modes to run (default
  --native-io,--pandas-io) plus extra CLI options, e.g. "--native-io,--gpus=2"
Writes a synthetic `{name}.mappings.bed` + header-only BAM (SURVEY §8d generator), runs the CLI
in-process twice (`--native-io`, then `--pandas-io`) with `--timings`, checks the two output pairs
are byte-identical, and records the per-stage seconds from the `timings_s` line.
"""
import contextlib
import filecmp
import io
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from click.testing import CliRunner  # noqa: E402

from fslr_amd import bam_header, synth  # noqa: E402
from fslr_amd.main import pipeline  # noqa: E402


def main():
    n, lmax, seed, out_json = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    dist = sys.argv[5] if len(sys.argv) > 5 else 'uniform'
    flags = sys.argv[6].split(',') if len(sys.argv) > 6 else ['--native-io', '--pandas-io']
    modes = [f for f in flags if f in ('--native-io', '--pandas-io')]
    repeat = 'repeat' in flags                   # run each mode a second time in this process (warm rank pool)
    extra = [f for f in flags if f not in modes and f != 'repeat']
    if repeat:
        modes = [m for m in modes for _ in (0, 1)]
    td = tempfile.mkdtemp(dir=os.environ.get('TMPDIR', '/tmp'))
    t0 = time.perf_counter()
    s = synth.generate(n, lmax, seed, dist=dist)
    s.write_tsv(os.path.join(td, 'x.mappings.bed'))
    bam_header.write_bam_header(os.path.join(td, 'x.bwa_dodi.bam'), list(s.chrom_lengths.items()))
    del s
    res = {'n_reads': n, 'lmax': lmax, 'seed': seed, 'dist': dist, 'extra_args': extra, 'gen_s': time.perf_counter() - t0,
           'bed_bytes': os.path.getsize(os.path.join(td, 'x.mappings.bed'))}
    print(json.dumps(res), flush=True)
    outs = {}
    for rep, flag in enumerate(modes):
        key = flag.strip('-') + ('_2' if repeat and rep % 2 else '')
        od = os.path.join(td, key)
        os.makedirs(od)
        for f in ('x.mappings.bed', 'x.bwa_dodi.bam'):
            os.symlink(os.path.join(td, f), os.path.join(od, f))
        err = io.StringIO()
        t1 = time.perf_counter()
        with contextlib.redirect_stderr(err):
            r = CliRunner().invoke(pipeline, ['--name', 'x', '--out', od, '--ref', 'u.fa', '--primers', '21q1',
                                              '--skip-alignment', '--timings', flag] + extra, catch_exceptions=False)
        wall = time.perf_counter() - t1
        line = [ln for ln in (r.output + err.getvalue()).splitlines() if ln.startswith('timings_s')]
        res[key] = {'wall_s': wall, 'exit': r.exit_code, 'timings': line[-1] if line else None}
        outs[key] = od
        print(json.dumps(res[key]), flush=True)
    keys = list(outs)
    res['outputs_identical'] = None if len(keys) < 2 else all(
        filecmp.cmp(os.path.join(outs[keys[0]], f), os.path.join(outs[k], f), shallow=False)
        for k in keys[1:] for f in ('x.mappings.cluster.bed', 'x.mappings.representative.bed'))
    with open(out_json, 'w') as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res), flush=True)


if __name__ == '__main__':
    main()
