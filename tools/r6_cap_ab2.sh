#!/bin/bash
# Round 6: the replay A/B again (product library vs rv1 = the round-5 replay), with the cap tests, and the
# replay clock build (libfslr_hip_rclk.so, -DFSLR_REPLAY_CLOCK): where the largest components' loops wait.
# Usage: gpurun -- bash tools/r6_cap_ab2.sh TAG [SUITE=cap|full|none]
set -o pipefail
TAG=${1:-r6k}
SUITE=${2:-cap}
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
bash tools/cap_ab.sh $TAG main rv1 rclk || exit 1
grep "replay clock" $O/capab_rclk.log | tail -2
echo done
