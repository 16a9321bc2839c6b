#!/bin/bash
# Counter-free pair-stage edge output: smoke, sweep / cap / dist / config GPU tests, bench A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-slots}
mkdir -p $O
cd $R
( while sleep 50; do echo "tick $(date +%T)"; done ) &
TICK=$!
trap "kill $TICK" EXIT
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 200 python3 bench.py --cpu-sample-stride 0 --steps 20 > $O/bench_slots.json 2> $O/bench_slots.log || { tail -20 $O/bench_slots.log; exit 1; }
bash tools/bench_variants.sh ${1:-slots} "" noslot "" || exit 1
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "sweep or cap or dist or config or parity" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
