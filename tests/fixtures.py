"""Loaders for the committed golden fixtures (tests/golden/, written by make_golden.py)."""
import gzip
import io
import json
import os

import pandas as pd

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')

FIXTURES = sorted(d for d in os.listdir(GOLDEN)
                  if os.path.isfile(os.path.join(GOLDEN, d, 'meta.json')))


def meta(name):
    with open(os.path.join(GOLDEN, name, 'meta.json')) as fh:
        return json.load(fh)


def input_dir(name):
    m = meta(name)
    return os.path.join(GOLDEN, m.get('input_from') or name)


def input_bed_text(name):
    with gzip.open(os.path.join(input_dir(name), 'input.mappings.bed.gz'), 'rt') as fh:
        return fh.read()


def input_bed(name):
    return pd.read_csv(io.StringIO(input_bed_text(name)), sep='\t')


def input_bam(name):
    return os.path.join(input_dir(name), 'input.bwa_dodi.bam')


def expected_text(name, which):
    p = os.path.join(GOLDEN, name, f'expected.{which}.bed.gz')
    if not os.path.exists(p):
        return None
    with gzip.open(p, 'rt') as fh:
        return fh.read()


def stage(name):
    p = os.path.join(GOLDEN, name, 'stage.json.gz')
    if not os.path.exists(p):
        return None
    with gzip.open(p, 'rt') as fh:
        return json.load(fh)


def cli_options(name):
    """Parse the fixture's CLI args into keyword options (defaults of main.py:33-37)."""
    kw = dict(overlap=0.8, jaccard_cutoffs='1,1,0.66,0.66,0.66,0.5', qlen_diff=0.04, n_alignment_diff=0.25,
              cluster_mask='subtelomere', filter_false=False)
    it = iter(meta(name)['args'])
    for a in it:
        key = a.lstrip('-').replace('-', '_')
        if key == 'filter_false':
            kw['filter_false'] = True
        else:
            v = next(it)
            kw[key] = float(v) if key in ('overlap', 'qlen_diff', 'n_alignment_diff') else v
    return kw


def kats():
    with gzip.open(os.path.join(GOLDEN, 'kats.json.gz'), 'rt') as fh:
        return json.load(fh)
