#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6t
mkdir -p $O
cd $R
( while sleep 50; do echo "tick $(date +%T)"; done ) &
TICK=$!
trap "kill $TICK" EXIT
timeout -k 10 600 python -u -m pytest tests/ --maxfail=1 -q --timeout 300 --timeout-method thread -m gpu -k "cap or config5 or dist or multi or shard" > $O/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 600 python3 -u tools/shard_cap_timing.py --worlds 8 --reps 3 > $O/capmodel.jsonl 2> $O/capmodel.log || { echo "capmodel failed"; tail -20 $O/capmodel.log; exit 1; }
grep -v "^fslr" $O/capmodel.log | tail -3
echo done
