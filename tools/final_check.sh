#!/bin/bash
# Long-read parity + kernel-trace stats + PMC traffic of the default bench (GPU box, repo root).
# Usage: bash tools/final_check.sh TAG
TAG=${1:-r02f}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_long.py tests/test_gpu_parity.py -k "long" -x -v --timeout 120 --timeout-method thread > $O/pytest_long.log 2>&1 || { tail -40 $O/pytest_long.log; exit 1; }
tail -3 $O/pytest_long.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --cpu-sample-stride 0 > $O/prof_bench.json 2> $O/prof.log || { tail -20 $O/prof.log; exit 1; }
cd $R
OUT=gpurun_out/$TAG/pmc bash tools/pmc.sh || exit 1
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.log || { tail -20 $O/bench.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); r=d['roofline']; print('value %.4e ms/step %.3f frac %.3f traffic %s' % (d['value'], d['ms_per_step'], r['frac'], r['traffic']))"
