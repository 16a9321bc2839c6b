#!/bin/bash
# One GPU iteration (repo root, via gpurun): GPU tests matching K -> bench line -> rocprof kernel table.
# Usage: bash tools/gpu_iter.sh TAG [pytest -k expression]
TAG=${1:-it}
K=${2:-"sweep or config or dist or kat"}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "$K" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --cpu-sample-stride 0 > $O/bench.json 2> $O/bench.log || { tail -20 $O/bench.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print('value %.4e ms/step %.3f' % (d['value'], d['ms_per_step']), d['roofline'].get('phase_ms_last_step'))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 1 --cpu-sample-stride 0 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
cd $R
python3 - "$(find $O/prof -name 'run_kernel_stats.csv' | head -1)" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:14]:
    print(f"{float(r['AverageNs'])/1000:9.1f} us  x{r['Calls']:>4}  {r['Name'][:90]}")
PY
