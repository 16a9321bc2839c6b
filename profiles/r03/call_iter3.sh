#!/bin/bash
# round-3 iteration: sweep-engine parity tests, long reads, then a short bench + kernel stats
# usage: bash tools/gpu_iter3.sh TAG ["pytest -k expression"]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-it}
K=${2:-sweep}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_long.py -x -q --timeout 300 \
    --timeout-method thread -m gpu -k "$K" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --cpu-sample-stride 0 > $O/bench.json 2> $O/bench.log || exit 1
python3 -c "import json,sys; d=json.load(open('$O/bench.json')); print('value %.4g ms/step %.4f' % (d['value'], d['ms_per_step']))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
    python3 $R/bench.py --steps 10 --warmup 2 --cpu-sample-stride 0 > $O/prof_bench.json 2> $O/prof.log || exit 1
cd $R
python3 - $O/prof/run_kernel_stats.csv <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:14]:
    print(f"{float(r['AverageNs'])/1000:9.1f} us  x{r['Calls']:>4}  {r['Name'][:80]}")
PY
