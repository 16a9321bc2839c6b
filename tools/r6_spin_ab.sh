#!/bin/bash
# Round 6: the default bench line with the step's two host readbacks polling the stream before the
# blocking wait (FSLR_SPIN_SYNC=1, the default) against the blocking wait alone (0), alternated 3 times.
# Usage: gpurun -- bash tools/r6_spin_ab.sh TAG
set -o pipefail
TAG=${1:-r6zj}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
for k in 1 2 3; do
  for v in 1 0; do
    FSLR_SPIN_SYNC=$v timeout -k 10 300 python3 bench.py > $O/bench_spin${v}_$k.json 2> $O/bench_spin${v}_$k.log \
        || { echo "bench $v $k failed"; tail -20 $O/bench_spin${v}_$k.log; exit 1; }
    python3 -c "import json; d=json.load(open('$O/bench_spin${v}_$k.json')); print('spin$v $k', d['ms_per_step'], d['value'], d['roofline']['kernel_ms'], d['config'].get('cold_step_ms'))"
  done
done
echo done
