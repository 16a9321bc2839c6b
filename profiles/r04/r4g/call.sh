#!/bin/bash
# Round-4: smoke, the GPU suite, the default bench, the per-rank models (cfg5 with the sharded cap at
# W = 2, 4, 8; cfg4 at W = 2, 4, 8), the cfg5 cap stage times on one GPU.
set -o pipefail
TAG=${1:-r4g}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
( while sleep 50; do echo "tick $(date +%T)"; done ) &
TICK=$!
trap "kill $TICK" EXIT
bline() { python3 -c "import json; d=json.load(open('$1')); r=d['roofline']; print('$2', 'ms/step %.4f' % d['ms_per_step'], r['kernel'], '%.4f' % r['kernel_ms'], [(x['kernel'], round(x['kernel_ms'],4)) for x in d.get('roofline_other_kernels', [])], {k: round(v, 3) for k, v in r['phase_ms_last_step'].items()}, d['config'].get('transfer'))"; }
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.log || { tail -20 $O/bench_default.log; exit 1; }
bline $O/bench_default.json default
FSLR_DEBUG_CAP=1 timeout -k 10 300 python3 tools/cfg5_cap.py --reps 3 > $O/cfg5_cap.json 2> $O/cfg5_cap.log || { tail -20 $O/cfg5_cap.log; exit 1; }
grep "fslr: cap stage" $O/cfg5_cap.log | tail -6
python3 -c "import json; d=json.load(open('$O/cfg5_cap.json')); print('cfg5 rep_ms', d['rep_ms'], d.get('full_equal'))"
timeout -k 10 500 python3 tools/shard_cap_timing.py --worlds 2,4,8 --reps 3 > $O/shard_cap.jsonl 2> $O/shard_cap.log || { tail -20 $O/shard_cap.log; exit 1; }
grep -E "^W=|cap_local parts" $O/shard_cap.log
timeout -k 10 300 python3 tools/shard_timing.py --reads 1000000 --lmax 16 --seed 11 --worlds 1,2,4,8 > $O/shard_cfg4.jsonl 2> $O/shard_cfg4.log || { tail -20 $O/shard_cfg4.log; exit 1; }
grep -E "^W=" $O/shard_cfg4.log
echo done
