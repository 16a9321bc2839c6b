#!/bin/bash
# Round-4: rocprofv3 kernel table of the cfg5 one-GPU cap replay on the round's last sources.
set -o pipefail
TAG=${1:-r4s}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
( while sleep 50; do echo "tick $(date +%T)"; done ) &
TICK=$!
trap "kill $TICK" EXIT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/tools/cfg5_cap.py --reps 3 > $O/cfg5_cap_prof.json 2> $O/cfg5_cap_prof.log || { tail -10 $O/cfg5_cap_prof.log; exit 1; }
cd $R
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/cfg5_cap_kernel_stats.csv
python3 - $O/cfg5_cap_kernel_stats.csv <<'PY'
import csv, sys, re
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:30]:
    n = re.sub(r'^void ', '', r['Name'].replace('(anonymous namespace)::', '')); i = n.find('('); n = n[:i] if i > 0 else n
    print(f"{float(r['AverageNs'])/1000:9.1f} us  x{r['Calls']:>4}  {n[:90]}")
PY
echo done
