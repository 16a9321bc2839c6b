#!/bin/bash
# All GPU tests, rocprofv3 kernel trace of the default bench, then the bench line (GPU box, repo root).
# Usage: bash tools/full_check.sh TAG
TAG=${1:-full}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --cpu-sample-stride 0 > $O/prof_bench.json 2> $O/prof.log || { tail -20 $O/prof.log; exit 1; }
cd $R
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.log || { tail -20 $O/bench.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); r=d['roofline']; print('value %.4e ms/step %.3f frac %.3f traffic %s' % (d['value'], d['ms_per_step'], r['frac'], r['traffic']))"
