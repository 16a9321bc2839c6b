#!/bin/bash
# cfg5 cap replay: kernel stats of the replay (rocprofv3) and the timing JSON
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-capprof}
mkdir -p $O
( while sleep 50; do echo "tick $(date +%T)"; done ) &
TICK=$!
trap "kill $TICK" EXIT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
    python3 $R/tools/cfg5_cap.py --reps 2 > $O/cfg5_cap.json 2> $O/cfg5_cap.log || { tail -20 $O/cfg5_cap.log; exit 1; }
cd $R
python3 - $O/prof/run_kernel_stats.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r['TotalDurationNs']) for r in rows if 'cap' in r['Name'] or 'k_fill' in r['Name'])
print('cap kernels total ms', tot / 1e6)
for r in rows:
    if 'k_cap' in r['Name'] or 'k_fill' in r['Name']:
        print(f"{float(r['TotalDurationNs'])/1e6:8.2f} ms  x{r['Calls']:>4}  {r['Name'][:90]}")
PY
