#!/bin/bash
# Round 6: the sharded cap at cfg5 W = 8 (the cap / dist / config5 GPU tests, the per-rank model and a
# kernel trace of it).  Usage: gpurun -- bash tools/r6_capprof.sh TAG
set -o pipefail
TAG=${1:-r6v}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
( while sleep 50; do echo "tick $(date +%T)"; done ) &
TICK=$!
trap "kill $TICK" EXIT
timeout -k 10 600 python -u -m pytest tests/ --maxfail=1 -q --timeout 300 --timeout-method thread -m gpu -k "cap or config5 or dist or multi or shard" > $O/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 600 python3 -u tools/shard_cap_timing.py --worlds 8 --reps 3 > $O/capmodel.jsonl 2> $O/capmodel.log || { echo "capmodel failed"; tail -20 $O/capmodel.log; exit 1; }
grep -v "^fslr" $O/capmodel.log | tail -2
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/capprof -o run --output-format csv \
    -- python3 $R/tools/shard_cap_timing.py --worlds 8 --reps 2 > $O/capshard.jsonl 2> $O/capshard.log ) || { echo "capshard prof failed"; tail -5 $O/capshard.log; exit 1; }
f=$(find $O/capprof -name 'run_kernel_stats.csv' | head -1); cp $f $O/capshard_kernel_stats.csv
f=$(find $O/capprof -name 'run_kernel_trace.csv' | head -1); cp $f $O/capshard_kernel_trace.csv
rm -rf $O/capprof
echo done
