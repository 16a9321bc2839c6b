#!/bin/bash
# Round-4 iteration: smoke, sweep tests, spill diagnostics, bench, rocprof of the bench, the cfg5 cap
# replay under rocprof (kernel table), stops at the first failure.
set -o pipefail
TAG=${1:-r4b}
K=${2:-"not slow and (sweep or repeat or cap)"}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
( while sleep 50; do echo "tick $(date +%T)"; done ) &
TICK=$!
trap "kill $TICK" EXIT
ktab() {
python3 - "$1" <<'PY'
import csv, sys, re
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:int(sys.argv[2]) if len(sys.argv) > 2 else 26]:
    n = r['Name'].replace('(anonymous namespace)::', '')
    n = re.sub(r'^void ', '', n); i = n.find('('); n = n[:i] if i > 0 else n
    print(f"{float(r['AverageNs'])/1000:9.1f} us  x{r['Calls']:>4}  tot {float(r['TotalDurationNs'])/1e6:8.3f} ms  {n[:80]}")
PY
}
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
FSLR_DEBUG_SPILL=1 timeout -k 10 240 python3 bench.py --steps 2 --warmup 1 --cpu-sample-stride 0 > $O/bench_spill.json 2> $O/bench_spill.log || { tail -20 $O/bench_spill.log; exit 1; }
grep "fslr: pair stage" $O/bench_spill.log | sort | uniq -c | head -5
timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.log || { tail -20 $O/bench.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); r=d['roofline']; print('value %.3e ms/step %.4f' % (d['value'], d['ms_per_step'])); print('roof', r['kernel'], '%.4f ms frac %.4f' % (r['kernel_ms'], r['frac']), [(x['kernel'], round(x['kernel_ms'],4)) for x in d['roofline_other_kernels']]); print(r['phase_ms_last_step'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --cpu-sample-stride 0 > $O/prof_bench.json 2> $O/prof.log || { tail -5 $O/prof.log; exit 1; }
ktab "$(find $O/prof -name 'run_kernel_stats.csv' | head -1)"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof5 -o run --output-format csv -- python3 $R/tools/cfg5_cap.py --reps 2 > $O/cfg5_cap.json 2> $O/cfg5_cap.log || { tail -20 $O/cfg5_cap.log; exit 1; }
cd $R
python3 -c "import json; d=json.load(open('$O/cfg5_cap.json')); print('cfg5 rep_ms', d['rep_ms'], 'query_ms', d['query_ms'], d.get('full_equal'))"
ktab "$(find $O/prof5 -name 'run_kernel_stats.csv' | head -1)" 45
echo done
