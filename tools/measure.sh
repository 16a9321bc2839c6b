#!/bin/bash
# One measurement pass on the GPU box (repo root, via gpurun):
#   default bench line -> rocprofv3 kernel stats of a short bench -> PMC traffic passes.
# Usage: bash tools/measure.sh TAG    (outputs under gpurun_out/TAG)
set -eo pipefail
TAG=${1:-m}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.log
python3 - $O/bench.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
r = d['roofline']
print('value %.3e %s  ms/step %.3f  kernel_ms %.3f  frac %.3f  algo %.2f GB' % (
    d['value'], d['unit'], d['ms_per_step'], r['kernel_ms'], r['frac'], r['algo_bytes_per_launch'] / 1e9))
print('cpu', json.dumps(d['cpu_baseline'])[:400])
PY
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
    python3 $R/bench.py --steps 5 --warmup 1 --cpu-sample-stride 0 > $O/prof.log 2>&1
cd $R
f=$(find $O/prof -name "run_kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:12]:
    print(f"{float(r['AverageNs'])/1000:9.1f} us  x{r['Calls']:>4}  {r['Name'][:90]}")
PY
OUT=gpurun_out/$TAG/pmc bash tools/pmc.sh
