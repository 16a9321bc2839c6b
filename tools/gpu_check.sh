#!/bin/bash
# One GPU-box pass after a kernel change (run from the repo root via gpurun):
#   parity tests -> section split (prof build) -> bench -> rocprofv3 kernel stats
# Usage: bash tools/gpu_check.sh TAG [extra pytest args]
set -e
TAG=${1:-chk}
shift || true
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 400 python -m pytest tests -m gpu -x -q "$@" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
if [ -f fslr_amd/libfslr_hip_prof.so ]; then
  timeout -k 10 300 python tools/sections.py > $O/sections.json 2> $O/sections.log
fi
timeout -k 10 300 python bench.py --cpu-sample-stride 0 > $O/bench.json 2> $O/bench.log
cat $O/bench.json | python -c "import json,sys; d=json.load(sys.stdin); print('ms/step', d['ms_per_step'], 'pairs/s %.3e' % d['value'], 'kernel_ms', d['roofline']['kernel_ms'], d['roofline']['phase_ms_last_step'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 1 --cpu-sample-stride 0 > $O/prof.log 2>&1
cd $R
f=$(find $O/prof -name "run_kernel_stats.csv" | head -1)
python - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:12]:
    print(f"{float(r['AverageNs'])/1000:9.1f} us  x{r['Calls']:>4}  {r['Name'][:90]}")
PY
