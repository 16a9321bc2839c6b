#!/bin/bash
# What the driver runs at round end: the whole GPU suite, smoke(), the default bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-roundend}
mkdir -p $O
cd $R
( while sleep 50; do echo "tick $(date +%T)"; done ) &
TICK=$!
trap "kill $TICK" EXIT
timeout -k 10 1000 python -u -m pytest tests/ -x -q --timeout 600 --timeout-method thread -m gpu > $O/pytest_gpu.log 2>&1 \
    || { echo "gpu tests failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.log || { tail -20 $O/bench.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); r=d['roofline']; c=d['cpu_baseline']; print('value %.4e ms/step %.3f cold %s kernel %s frac %.3f traffic %s cpu %s' % (d['value'], d['ms_per_step'], d['config'].get('cold_step_ms'), r['kernel'], r['frac'], r['traffic'], c and c['value']))"
