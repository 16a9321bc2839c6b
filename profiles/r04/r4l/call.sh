#!/bin/bash
# Round-4: one-GPU cap with the segmented slot sort and per-read slot ranges (suite, cfg5 cap stage
# times, A/B against the global sort), the sharded cap model at W=8, PMC of the sweep kernels on the
# current sources.
set -o pipefail
TAG=${1:-r4l}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
( while sleep 50; do echo "tick $(date +%T)"; done ) &
TICK=$!
trap "kill $TICK" EXIT
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
FSLR_DEBUG_CAP=1 timeout -k 10 300 python3 tools/cfg5_cap.py --reps 3 > $O/cfg5_cap_dbg.json 2> $O/cfg5_cap_dbg.log || { tail -20 $O/cfg5_cap_dbg.log; exit 1; }
grep -E "stage|rep " $O/cfg5_cap_dbg.log | tail -8
timeout -k 10 300 python3 tools/cfg5_cap.py --reps 3 > $O/cfg5_cap.json 2> $O/cfg5_cap.log || { tail -20 $O/cfg5_cap.log; exit 1; }
grep -E "rep " $O/cfg5_cap.log | tail -2
FSLR_CAP_SLOTSORT=global timeout -k 10 300 python3 tools/cfg5_cap.py --reps 3 > $O/cfg5_cap_global.json 2> $O/cfg5_cap_global.log || { tail -20 $O/cfg5_cap_global.log; exit 1; }
grep -E "rep " $O/cfg5_cap_global.log | tail -2
timeout -k 10 400 python3 tools/shard_cap_timing.py --worlds 8 --reps 2 > $O/shard_cap_w8.jsonl 2> $O/shard_cap_w8.log || { tail -20 $O/shard_cap_w8.log; exit 1; }
grep -E "^W=|parts" $O/shard_cap_w8.log
OUT=gpurun_out/$TAG/pmc timeout -k 10 600 bash tools/pmc.sh > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
tail -2 $O/pmc.log
echo done
