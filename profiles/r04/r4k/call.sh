#!/bin/bash
# Round-4: the one-GPU cap replay over the edge list's runs (closure by frontier, T's runs classified
# in place): GPU suite, cfg5 cap stage times and clean times, bench.
set -o pipefail
TAG=${1:-r4k}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
( while sleep 50; do echo "tick $(date +%T)"; done ) &
TICK=$!
trap "kill $TICK" EXIT
bline() { python3 -c "import json; d=json.load(open('$1')); r=d['roofline']; print('$2', 'ms/step %.4f' % d['ms_per_step'], r['kernel'], '%.4f' % r['kernel_ms'], [(x['kernel'], round(x['kernel_ms'],4)) for x in d.get('roofline_other_kernels', [])], {k: round(v, 3) for k, v in r['phase_ms_last_step'].items() if k in ('index_ms','query_ms','sweep_count_ms','sweep_sort_ms','sweep_pairs_ms')})"; }
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
FSLR_DEBUG_CAP=1 timeout -k 10 300 python3 tools/cfg5_cap.py --reps 3 > $O/cfg5_cap_dbg.json 2> $O/cfg5_cap_dbg.log || { tail -20 $O/cfg5_cap_dbg.log; exit 1; }
grep -E "grouped|stage|rep " $O/cfg5_cap_dbg.log | tail -12
timeout -k 10 300 python3 tools/cfg5_cap.py --reps 3 > $O/cfg5_cap.json 2> $O/cfg5_cap.log || { tail -20 $O/cfg5_cap.log; exit 1; }
grep -E "rep " $O/cfg5_cap.log | tail -3
FSLR_CAP_RUNS=0 timeout -k 10 300 python3 tools/cfg5_cap.py --reps 3 > $O/cfg5_cap_full.json 2> $O/cfg5_cap_full.log || { tail -20 $O/cfg5_cap_full.log; exit 1; }
grep -E "rep " $O/cfg5_cap_full.log | tail -3
timeout -k 10 240 python3 bench.py --steps 30 --warmup 5 --cpu-sample-stride 0 > $O/bench.json 2> $O/bench.log || { tail -20 $O/bench.log; exit 1; }
bline $O/bench.json bench
echo done
