#!/bin/bash
# Round 6: the edge-cap replay with its loads ahead (k_cap_replay / replay_read_ahead) against the
# round-5 replay (libfslr_hip_rv1.so, -DFSLR_CAP_REPLAY_V1): the GPU suite on the product library, the
# cfg5 one-GPU per-stage times of both (tools/cap_ab.sh), then the W = 8 cap model of the product library.
# Usage: gpurun -- bash tools/r6_cap_ab.sh TAG [SUITE=full|cap|none]
set -o pipefail
TAG=${1:-r6j}
SUITE=${2:-full}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
( while sleep 50; do echo "tick $(date +%T)"; done ) &
TICK=$!
trap "kill $TICK" EXIT
if [ "$SUITE" != none ]; then
  K=()
  [ "$SUITE" = cap ] && K=(-k "cap or config5 or zdcap or long")
  timeout -k 10 900 python -u -m pytest tests/ --maxfail=1 -q --timeout 300 --timeout-method thread -m gpu "${K[@]}" \
      > $O/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -40 $O/pytest_gpu.log; exit 1; }
  tail -1 $O/pytest_gpu.log
fi
bash tools/cap_ab.sh $TAG main rv1 || exit 1
timeout -k 10 600 python3 -u tools/shard_cap_timing.py --worlds 8 --reps 3 > $O/capmodel.jsonl 2> $O/capmodel.log \
    || { echo "capmodel failed"; tail -20 $O/capmodel.log; exit 1; }
grep -v "^fslr" $O/capmodel.log | tail -3
echo done
