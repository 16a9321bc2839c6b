#!/bin/bash
# PMC passes (separate rocprofv3 runs, no traces) for the kernels matching REGEX on a short bench.
# Usage (GPU box, repo root): OUT=gpurun_out/pmcX REGEX='k_sweep' bash tools/pmc_kernels.sh [bench args]
set -e
OUT=${OUT:-gpurun_out/pmc}
REGEX=${REGEX:-k_sweep}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $ROOT/$OUT
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE" "SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_BUSY_CYCLES" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-include-regex "$REGEX" -d $ROOT/$OUT/p$i -o pmc \
      --output-format csv -- python3 $ROOT/bench.py --steps 2 --warmup 1 --cpu-sample-stride 0 "$@" \
      > $ROOT/$OUT/p$i.log 2>&1
done
cd $ROOT
python3 - $ROOT/$OUT <<'PY'
import csv, glob, os, sys
from collections import defaultdict
vals = defaultdict(lambda: defaultdict(list))
for path in glob.glob(os.path.join(sys.argv[1], '**', '*counter_collection.csv'), recursive=True):
    for row in csv.DictReader(open(path)):
        vals[row['Kernel_Name'][:60]][row['Counter_Name']].append(float(row['Counter_Value']))
for k, d in vals.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f'   {c:22s} {sum(v) / len(v):16.1f}  (n={len(v)})')
PY
