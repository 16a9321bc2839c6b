#!/bin/bash
# Round 6: the default bench line with the timed steps carrying the pair-stage kernel's events alone
# (profiling level 3) against both kernels' events (FSLR_BENCH_EVENTS=both, level 2), alternated 3 times.
# Usage: gpurun -- bash tools/r6_events_ab.sh TAG
set -o pipefail
TAG=${1:-r6zi}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
for k in 1 2 3; do
  for v in stage both; do
    FSLR_BENCH_EVENTS=$v timeout -k 10 300 python3 bench.py > $O/bench_${v}_$k.json 2> $O/bench_${v}_$k.log \
        || { echo "bench $v $k failed"; tail -20 $O/bench_${v}_$k.log; exit 1; }
    python3 -c "import json; d=json.load(open('$O/bench_${v}_$k.json')); print('$v $k', d['ms_per_step'], d['value'], d['roofline']['kernel_ms'])"
  done
done
echo done
