#!/bin/bash
# Round-4: the cap slots sorted per read in LDS (suite, cfg5 A/B against the segmented radix sort,
# stage times), the sharded model at W=8.
set -o pipefail
TAG=${1:-r4n}
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
grep -E "stage|rep " $O/cfg5_cap_dbg.log | tail -11
timeout -k 10 300 python3 tools/cfg5_cap.py --reps 3 > $O/cfg5_cap.json 2> $O/cfg5_cap.log || { tail -20 $O/cfg5_cap.log; exit 1; }
grep -E "rep " $O/cfg5_cap.log | tail -2
FSLR_CAP_SLOTSORT=seg timeout -k 10 300 python3 tools/cfg5_cap.py --reps 3 > $O/cfg5_cap_seg.json 2> $O/cfg5_cap_seg.log || { tail -20 $O/cfg5_cap_seg.log; exit 1; }
grep -E "rep " $O/cfg5_cap_seg.log | tail -2
timeout -k 10 400 python3 tools/shard_cap_timing.py --worlds 8 --reps 3 > $O/shard_cap_w8.jsonl 2> $O/shard_cap_w8.log || { tail -20 $O/shard_cap_w8.log; exit 1; }
grep -E "^W=|parts" $O/shard_cap_w8.log
echo done
