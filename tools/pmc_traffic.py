#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (tools/pmc.sh) into per-launch HBM traffic of the pair kernel.

    python tools/pmc_traffic.py gpurun_out/pmc [-o profiles/r01/pmc_traffic.json]

Reads every */pmc_counter_collection.csv under the directory, keeps the dispatches of the
named kernel, and averages each counter per dispatch.  HBM bytes per launch follow
/opt/skills/guides/MI355X_MICROARCH.md (HBM / rocprofv3 section):
  FETCH_SIZE, WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports 1/2 of the bytes of wide
  (16 B/lane) streaming reads.  Other widths are calibrated on known byte counts
  (tools/fetchcal.sh -> profiles/r06/fetch_calibration.json: 16-, 8- and 4-B/lane loads all read as
  0.500 of their bytes), and the kernel's correction is the calibrated one of its load widths; the
  uncorrected figure is kept beside it.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
from collections import defaultdict


CALIBRATION = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'profiles', 'r06',
                           'fetch_calibration.json')
# the global-load widths per lane of each kernel (all must be calibrated to apply the calibration):
# k_sweep<2>: 16-B records and gate ranges, 8-B gate words and slots, 4-B windows; k_sweep_pairs: 8-B
# entries (its 1-B read lengths are gathers that stay in L2)
LOAD_WIDTHS = {'k_sweep<2>': [16, 8, 4], 'k_sweep_pairs': [8], 'query_kernel<0, false>': [16, 8, 4]}


def collect(root, kernel):
    vals = defaultdict(list)
    dur = []
    for path in sorted(glob.glob(os.path.join(root, '**', '*counter_collection.csv'), recursive=True)):
        with open(path, newline='') as fh:
            for row in csv.DictReader(fh):
                if kernel not in row['Kernel_Name']:
                    continue
                vals[row['Counter_Name']].append(float(row['Counter_Value']))
                if row['Counter_Name'] in ('FETCH_SIZE', 'SQ_WAVES'):
                    dur.append((int(row['End_Timestamp']) - int(row['Start_Timestamp'])) * 1e-9)
    return {k: sum(v) / len(v) for k, v in vals.items()}, dur


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('root')
    ap.add_argument('--kernel', default='k_sweep<2>')
    ap.add_argument('-o', '--out', default=None)
    ap.add_argument('--source-hash', default=None, help='hash of the kernel sources the counters were taken on')
    ap.add_argument('--merge-into', default=None,
                    help='a JSON object keyed by kernel name (bench.py --traffic-json): set this kernel\'s entry')
    ap.add_argument('--calibration', default=CALIBRATION,
                    help='tools/fetch_calibration.py output: FETCH_SIZE / WRITE_SIZE per known byte, per width')
    args = ap.parse_args()
    c, dur = collect(args.root, args.kernel)
    if 'FETCH_SIZE' not in c:
        raise SystemExit(f'no FETCH_SIZE rows for {args.kernel} under {args.root}')
    fetch = c['FETCH_SIZE'] * 1024.0
    write = c.get('WRITE_SIZE', 0.0) * 1024.0
    # the read correction from the calibration of this kernel's load widths (every width it loads must
    # be calibrated, and they must agree: FETCH_SIZE cannot be split by width)
    widths = LOAD_WIDTHS.get(args.kernel)
    cal = json.load(open(args.calibration)) if args.calibration and os.path.exists(args.calibration) else None
    factor, basis = None, None
    if cal and widths:
        ratios = [cal['ratio_by_width']['read'].get(str(w)) for w in widths]
        if all(r for r in ratios) and max(ratios) - min(ratios) < 0.01 * max(ratios):
            factor = 1.0 / (sum(ratios) / len(ratios))
            basis = (f'{os.path.relpath(args.calibration)}: FETCH_SIZE = {sum(ratios) / len(ratios):.4f} x the bytes '
                     f'of {"/".join(str(w) for w in widths)}-B/lane streaming loads (a 1 GiB buffer each)')
    if factor is None:
        factor = 2.0
        basis = 'MI355X_MICROARCH.md: FETCH_SIZE x2 on gfx950 for 16-B/lane reads (uncalibrated for other widths)'
    out = {
        'kernel': args.kernel,
        'hbm_bytes_per_launch': factor * fetch + write,
        'fetch_bytes_raw': fetch,
        'fetch_correction_factor': factor,
        'fetch_bytes_corrected': factor * fetch,
        'write_bytes': write,
        'load_widths_bytes': widths,
        'pmc_pass_launch_s_mean': (sum(dur) / len(dur)) if dur else None,
        'counters_mean_per_dispatch': c,
        'correction': basis + '; WRITE_SIZE as is (calibrated 1.00 for 8- and 16-B streaming stores)',
        'source_hash': args.source_hash,
    }
    if 'TCC_HIT_sum' in c and 'TCC_MISS_sum' in c:
        out['l2_hit_rate'] = c['TCC_HIT_sum'] / max(1.0, c['TCC_HIT_sum'] + c['TCC_MISS_sum'])
    if 'SQ_INSTS_VALU' in c and c.get('GRBM_GUI_ACTIVE'):
        # VALU issue: a wave64 VALU instruction takes 2 cycles of a SIMD (MI355X_MICROARCH.md), 1024
        # SIMDs; GRBM_GUI_ACTIVE sums the 8 XCDs' busy cycles, so / 8 is the launch's cycles
        cyc = c['GRBM_GUI_ACTIVE'] / 8.0
        out['valu_issue_frac'] = 2.0 * c['SQ_INSTS_VALU'] / (1024.0 * cyc)
    if 'SQ_WAVE_CYCLES' in c:
        wc = max(1.0, c['SQ_WAVE_CYCLES'])
        out['wave_cycle_split'] = {k: c.get(k, 0.0) / wc for k in ('SQ_WAIT_ANY', 'SQ_WAIT_INST_ANY',
                                                                  'SQ_ACTIVE_INST_ANY')}
    text = json.dumps(out, indent=1)
    if args.merge_into:
        allk = {}
        if os.path.exists(args.merge_into):
            with open(args.merge_into) as fh:
                allk = json.load(fh)
            if 'kernel' in allk:                        # an older single-kernel summary
                allk = {allk['kernel']: allk}
        allk[args.kernel] = out
        with open(args.merge_into, 'w') as fh:
            fh.write(json.dumps(allk, indent=1) + '\n')
    if args.out:
        with open(args.out, 'w') as fh:
            fh.write(text + '\n')
    print(text)


if __name__ == '__main__':
    main()
