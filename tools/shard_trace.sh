#!/bin/bash
# Kernel trace of the chromosome-split sweep at one world size (repo root, via gpurun):
#   bash tools/shard_trace.sh TAG W [READS]
# rocprofv3 --kernel-trace over tools/shard_timing.py --worlds W; the per-dispatch CSV lets
# tools/trace_phases.py split one rank's partition / evaluation into kernels.
TAG=${1:-st}
W=${2:-8}
N=${3:-1000000}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
  python3 $R/tools/shard_timing.py --reads $N --lmax 16 --worlds $W --reps 3 > $O/shard.json 2> $O/shard.log || { tail -5 $O/shard.log; exit 1; }
tail -3 $O/shard.log
