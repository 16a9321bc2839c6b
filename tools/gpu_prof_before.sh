#!/bin/bash
# kernel trace + PMC passes of k_sweep_pairs on the current tree (round-3 "before" profile)
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3_before
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
    python3 $R/bench.py --steps 10 --warmup 2 --cpu-sample-stride 0 > $O/bench.json 2> $O/bench.log
cd $R
OUT=gpurun_out/r3_before/pmc REGEX='k_sweep_pairs' bash tools/pmc_kernels.sh > $O/pmc_summary.txt 2>&1
