#!/bin/bash
# Round-4: the restricted cap gather — GPU suite, cfg5 W=8 per-rank model with stage timers, bench.
set -o pipefail
TAG=${1:-r4i}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
( while sleep 50; do echo "tick $(date +%T)"; done ) &
TICK=$!
trap "kill $TICK" EXIT
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
FSLR_DEBUG_CAP=1 timeout -k 10 400 python3 tools/shard_cap_timing.py --worlds 8 --reps 2 > $O/shard_cap_w8.jsonl 2> $O/shard_cap_w8.log || { tail -20 $O/shard_cap_w8.log; exit 1; }
grep -E "restricted|^W=|parts" $O/shard_cap_w8.log
python3 - $O/shard_cap_w8.log <<'PY'
import re, sys, collections
mx = collections.OrderedDict()
for line in open(sys.argv[1]):
    m = re.match(r'fslr: cap stage (.+?)\s+([0-9.]+) ms', line)
    if m:
        k = m.group(1).strip(); mx.setdefault(k, []).append(float(m.group(2)))
for k, v in mx.items():
    print(f'{k:16s} n={len(v):3d} max={max(v):8.3f} median={sorted(v)[len(v)//2]:8.3f}')
PY
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.log || { tail -20 $O/bench.log; exit 1; }
cat $O/bench.json | cut -c1-600
echo done
