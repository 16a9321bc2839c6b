#!/bin/bash
# Round-4: A/B of the sweep's tile-header prefetch and the pair stage's early next window / L_B by
# position (compile-time variants, FSLR_LIB), then the GPU suite on the default build.
set -o pipefail
TAG=${1:-r4j}
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
for v in base pf1 pf2 pf3 pf1w6 pf3w6 early lbpos elb base2; do
  case $v in base|base2) L="";; *) L="FSLR_LIB=$R/fslr_amd/libfslr_hip_$v.so";; esac
  env $L timeout -k 10 240 python3 bench.py --steps 30 --warmup 5 --cpu-sample-stride 0 > $O/bench_$v.json 2> $O/bench_$v.log || { tail -20 $O/bench_$v.log; exit 1; }
  bline $O/bench_$v.json $v
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
echo done
