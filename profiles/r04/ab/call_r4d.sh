#!/bin/bash
# Round-4: smoke, the whole GPU suite, bench A/B (sweep chunk map x pair stage), the sharded cap
# timing model at cfg5 W=8, the cfg5 cap replay under rocprof and its round-3 variant.  Stops at the
# first failure.
set -o pipefail
TAG=${1:-r4d}
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
for v in default map_stride legacy both; do
  case $v in
    default) E="";; map_stride) E="FSLR_SWEEP_MAP=stride";; legacy) E="FSLR_PAIR_STAGE=legacy";; both) E="FSLR_SWEEP_MAP=stride FSLR_PAIR_STAGE=legacy";;
  esac
  env $E timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 --cpu-sample-stride 0 > $O/bench_$v.json 2> $O/bench_$v.log || { tail -20 $O/bench_$v.log; exit 1; }
  bline $O/bench_$v.json $v
done
timeout -k 10 400 python3 tools/shard_cap_timing.py --worlds 8 --reps 3 > $O/shard_cap_w8.jsonl 2> $O/shard_cap_w8.log || { tail -20 $O/shard_cap_w8.log; exit 1; }
tail -2 $O/shard_cap_w8.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof5 -o run --output-format csv -- python3 $R/tools/cfg5_cap.py --reps 2 > $O/cfg5_cap.json 2> $O/cfg5_cap.log || { tail -20 $O/cfg5_cap.log; exit 1; }
cd $R
python3 -c "import json; d=json.load(open('$O/cfg5_cap.json')); print('cfg5 rep_ms', d['rep_ms'], 'query_ms', d['query_ms'], d.get('full_equal'))"
ktab "$(find $O/prof5 -name 'run_kernel_stats.csv' | head -1)" 40
FSLR_CAP_CLOSURE=rounds FSLR_CAP_REPLAY=components timeout -k 10 300 python3 tools/cfg5_cap.py --reps 2 > $O/cfg5_cap_r3.json 2> $O/cfg5_cap_r3.log || { tail -20 $O/cfg5_cap_r3.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/cfg5_cap_r3.json')); print('cfg5 r3-variant rep_ms', d['rep_ms'], d.get('full_equal'))"
echo done
