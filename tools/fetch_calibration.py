#!/usr/bin/env python3
"""FETCH_SIZE / WRITE_SIZE per known byte, per access width (tools/fetchcal.sh on the GPU box).

    python tools/fetch_calibration.py gpurun_out/cal -o profiles/r06/fetch_calibration.json

For each kernel of tools/microbench/fetchcal.hip (one access width, a 1 GiB buffer streamed once):
fetch_ratio = FETCH_SIZE bytes / algorithmic read bytes, write_ratio = WRITE_SIZE bytes / algorithmic
write bytes, and the HBM rate from the kernel trace.  tools/pmc_traffic.py divides a kernel's counters by
the ratio of its dominant access width (MI355X_MICROARCH.md: 'calibrate on a known byte count').
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def counters(root):
    vals = defaultdict(lambda: defaultdict(list))
    for path in glob.glob(os.path.join(root, '**', '*counter_collection.csv'), recursive=True):
        with open(path, newline='') as fh:
            for row in csv.DictReader(fh):
                name = row['Kernel_Name'].split('(')[0].replace('void ', '').strip()
                vals[name][row['Counter_Name']].append(float(row['Counter_Value']))
    return {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in vals.items()}


def durations(root):
    out = {}
    for path in glob.glob(os.path.join(root, '**', '*kernel_stats.csv'), recursive=True):
        with open(path, newline='') as fh:
            for row in csv.DictReader(fh):
                name = row['Name'].split('(')[0].replace('void ', '').strip()
                out[name] = float(row['AverageNs']) * 1e-9
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('root')
    ap.add_argument('-o', '--out', required=True)
    a = ap.parse_args()
    known = json.load(open(os.path.join(a.root, 'known.json')))['kernels']
    c = counters(a.root)
    d = durations(a.root)
    res = {}
    for k, kb in known.items():
        cc = c.get(k, {})
        f = cc.get('FETCH_SIZE')
        w = cc.get('WRITE_SIZE')
        e = dict(kb)
        if kb['read'] and f is not None:
            e['fetch_bytes'] = f * 1024.0
            e['fetch_ratio'] = f * 1024.0 / kb['read']
        if kb['write'] and w is not None:
            e['write_bytes'] = w * 1024.0
            e['write_ratio'] = w * 1024.0 / kb['write']
        if k in d:
            e['seconds'] = d[k]
            e['gbs'] = (kb['read'] + kb['write']) / d[k] / 1e9
        res[k] = e
    by_width = {'read': {}, 'write': {}}
    for k, e in res.items():
        if 'fetch_ratio' in e:
            by_width['read'][str(e['width'])] = e['fetch_ratio']
        if 'write_ratio' in e and 'run' not in e:
            by_width['write'][str(e['width'])] = e['write_ratio']
        if 'write_ratio' in e and 'run' in e:
            by_width['write'][f"{e['width']}_runs{e['run']}"] = e['write_ratio']
    out = {'kernels': res, 'ratio_by_width': by_width,
           'method': 'tools/microbench/fetchcal.hip: each kernel streams a 1 GiB buffer (4x the Infinity Cache) '
                     'once with one access width; ratio = counter bytes (KiB x 1024) / algorithmic bytes'}
    with open(a.out, 'w') as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(by_width))


if __name__ == '__main__':
    main()
