#!/usr/bin/env python3
"""Run the product CLI on a golden fixture several times (both I/O modes) and print the first lines
that differ from the reference's expected outputs (diagnostics for tests/test_gpu_parity.py)."""
import os
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, 'tests'), os.path.join(REPO, 'tests', 'golden')]
import fixtures as fx  # noqa: E402
from test_gpu_parity import run_product_cli  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else 'capbind_1500'
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
for rep in range(reps):
    for io in ('--native-io', '--pandas-io'):
        with tempfile.TemporaryDirectory() as tmp:
            res = run_product_cli(name, tmp, io)
            for which in ('cluster', 'representative'):
                want = fx.expected_text(name, which).splitlines()
                got = open(os.path.join(tmp, f'fx.mappings.{which}.bed')).read().splitlines()
                bad = [(k, g, w) for k, (g, w) in enumerate(zip(got, want)) if g != w]
                print(f'rep {rep} {io} {which}: {len(got)} vs {len(want)} lines, {len(bad)} differ', flush=True)
                for k, g, w in bad[:4]:
                    print(f'   line {k}\n     got  {g}\n     want {w}')
