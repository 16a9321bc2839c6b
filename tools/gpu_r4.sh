#!/bin/bash
# Round-4 check on the box: smoke, the GPU tests matching K, the default bench line, its rocprof
# kernel table, then the cfg5 cap replay (timings + full-graph digests).  Stops at the first failure.
# Usage: bash tools/gpu_r4.sh TAG [pytest -k expression] [cfg5: 1|0]
set -o pipefail
TAG=${1:-r4}
K=${2:-"not slow"}
CFG5=${3:-1}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
( while sleep 50; do echo "tick $(date +%T)"; done ) &
TICK=$!
trap "kill $TICK" EXIT
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.log || { tail -20 $O/bench.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); r=d['roofline']; print('value %.3e ms/step %.4f' % (d['value'], d['ms_per_step'])); print('roof', r['kernel'], '%.4f ms frac %.4f' % (r['kernel_ms'], r['frac']), [(x['kernel'], round(x['kernel_ms'],4)) for x in d['roofline_other_kernels']]); print(r['phase_ms_last_step'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --cpu-sample-stride 0 > $O/prof_bench.json 2> $O/prof.log || { tail -5 $O/prof.log; exit 1; }
cd $R
python3 - "$(find $O/prof -name 'run_kernel_stats.csv' | head -1)" <<'PY'
import csv, sys, re
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:18]:
    n = re.sub(r'\(.*', '', r['Name'])[-70:]
    print(f"{float(r['AverageNs'])/1000:9.1f} us  x{r['Calls']:>4}  {n}")
PY
if [ "$CFG5" = 1 ]; then
  timeout -k 10 600 python3 tools/cfg5_cap.py --reps 3 > $O/cfg5_cap.json 2> $O/cfg5_cap.log || { tail -20 $O/cfg5_cap.log; exit 1; }
  python3 -c "import json; d=json.load(open('$O/cfg5_cap.json')); print('cfg5 rep_ms', d['rep_ms'], 'query_ms', d['query_ms'], d.get('full_equal'), d.get('sample_edges_equal'))"
fi
echo done
