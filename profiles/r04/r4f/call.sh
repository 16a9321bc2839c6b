#!/bin/bash
# Round-4: smoke, the GPU suite, the default bench, the cfg5 cap replay's stage times on one GPU and
# per rank of the sharded replay at W=8 (FSLR_DEBUG_CAP), and the sharded model's kernel table.
set -o pipefail
TAG=${1:-r4f}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
( while sleep 50; do echo "tick $(date +%T)"; done ) &
TICK=$!
trap "kill $TICK" EXIT
ktab() {
python3 - "$1" "$2" <<'PY'
import csv, sys, re
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:int(sys.argv[2]) if len(sys.argv) > 2 else 26]:
    n = r['Name'].replace('(anonymous namespace)::', '')
    n = re.sub(r'^void ', '', n); i = n.find('('); n = n[:i] if i > 0 else n
    print(f"{float(r['AverageNs'])/1000:9.1f} us  x{r['Calls']:>4}  tot {float(r['TotalDurationNs'])/1e6:8.3f} ms  {n[:80]}")
PY
}
bline() { python3 -c "import json; d=json.load(open('$1')); r=d['roofline']; print('$2', 'ms/step %.4f' % d['ms_per_step'], r['kernel'], '%.4f' % r['kernel_ms'], [(x['kernel'], round(x['kernel_ms'],4)) for x in d.get('roofline_other_kernels', [])], {k: round(v, 3) for k, v in r['phase_ms_last_step'].items()})"; }
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.log || { tail -20 $O/bench_default.log; exit 1; }
bline $O/bench_default.json default
FSLR_DEBUG_CAP=1 timeout -k 10 300 python3 tools/cfg5_cap.py --reps 3 > $O/cfg5_cap.json 2> $O/cfg5_cap.log || { tail -20 $O/cfg5_cap.log; exit 1; }
grep "fslr: cap" $O/cfg5_cap.log | tail -12
python3 -c "import json; d=json.load(open('$O/cfg5_cap.json')); print('cfg5 rep_ms', d['rep_ms'], d.get('full_equal'))"
timeout -k 10 400 python3 tools/shard_cap_timing.py --worlds 8 --reps 3 > $O/shard_cap_w8.jsonl 2> $O/shard_cap_w8.log || { tail -20 $O/shard_cap_w8.log; exit 1; }
tail -3 $O/shard_cap_w8.log
FSLR_DEBUG_CAP=1 timeout -k 10 400 python3 tools/shard_cap_timing.py --worlds 8 --reps 1 > $O/shard_cap_dbg.jsonl 2> $O/shard_cap_dbg.log || { tail -20 $O/shard_cap_dbg.log; exit 1; }
grep "fslr: cap stage" $O/shard_cap_dbg.log | sort -k4,5 | awk '{k=$4" "$5; if ($6 ~ /ms/) {v=$5} } {print}' | tail -5
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
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/profsh -o run --output-format csv -- python3 $R/tools/shard_cap_timing.py --worlds 8 --reps 1 > $O/shard_cap_prof.jsonl 2> $O/shard_cap_prof.log || { tail -5 $O/shard_cap_prof.log; exit 1; }
cd $R
ktab "$(find $O/profsh -name 'run_kernel_stats.csv' | head -1)" 45
echo done
