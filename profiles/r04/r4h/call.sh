#!/bin/bash
# Round-4: the sharded cap's per-rank stage times (FSLR_DEBUG_CAP) and the restricted-gather sizes at
# cfg5 W=8, the CLI at 2M reads x 1-64 Zipf (native I/O), PMC passes of the default sweep kernels.
set -o pipefail
TAG=${1:-r4h}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
( while sleep 50; do echo "tick $(date +%T)"; done ) &
TICK=$!
trap "kill $TICK" EXIT
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
FSLR_DEBUG_CAP=1 timeout -k 10 400 python3 tools/shard_cap_timing.py --worlds 8 --reps 2 > $O/shard_cap_dbg.jsonl 2> $O/shard_cap_dbg.log || { tail -20 $O/shard_cap_dbg.log; exit 1; }
grep -E "restricted|^W=" $O/shard_cap_dbg.log
python3 - $O/shard_cap_dbg.log <<'PY'
import re, sys, collections
mx = collections.OrderedDict()
for line in open(sys.argv[1]):
    m = re.match(r'fslr: cap stage (.+?)\s+([0-9.]+) ms', line)
    if m:
        k = m.group(1).strip(); mx.setdefault(k, []).append(float(m.group(2)))
for k, v in mx.items():
    print(f'{k:16s} n={len(v):3d} max={max(v):8.3f} median={sorted(v)[len(v)//2]:8.3f}')
PY
timeout -k 10 600 python3 tools/cli_io_timing.py 2000000 64 13 $O/cli_2m.json zipf --native-io > $O/cli_2m.log 2>&1 || { tail -20 $O/cli_2m.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/cli_2m.json')); print({k: v for k, v in d.items() if k not in ('extra_args',)})"
OUT=gpurun_out/$TAG/pmc timeout -k 10 600 bash tools/pmc.sh > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
tail -2 $O/pmc.log
python3 -c "import json; d=json.load(open('$O/pmc/traffic.json')); print(json.dumps(d)[:1500])"
echo done
