#!/bin/bash
# sweep GPU tests, then the default bench line (CPU baseline included) twice on this box
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-bd}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "sweep and not slow" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for k in 1 2; do
  timeout -k 10 400 python3 bench.py > $O/bench_$k.json 2> $O/bench_$k.log || { tail -20 $O/bench_$k.log; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$k.json')); r=d['roofline']; c=d['cpu_baseline']; print('value %.4e ms/step %.3f cold %.3f kernel %s %.4f ms frac %.3f traffic %s cpu %.3e' % (d['value'], d['ms_per_step'], d['config']['cold_step_ms'], r['kernel'], r['kernel_ms'], r['frac'], r['traffic'], c['value']))"
done
