#!/bin/bash
# Round-4 end measurements: the default bench (with the CPU baseline) and its rocprofv3 kernel table,
# the per-rank models with the sharded cap at W = 2, 4 (cfg5) and the uncapped cfg4 model.
set -o pipefail
TAG=${1:-r4m}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
( while sleep 50; do echo "tick $(date +%T)"; done ) &
TICK=$!
trap "kill $TICK" EXIT
bline() { python3 -c "import json; d=json.load(open('$1')); r=d['roofline']; print('$2', 'ms/step %.4f' % d['ms_per_step'], r['kernel'], '%.4f' % r['kernel_ms'], 'frac %.3f' % r['frac'], 'traffic', r.get('traffic'), 'valu', r.get('valu_issue_frac'), [(x['kernel'], round(x['kernel_ms'],4), round(x['frac'],3)) for x in d.get('roofline_other_kernels', [])], d.get('cpu_baseline', {}).get('value'))"; }
timeout -k 10 300 python3 bench.py > $O/bench_default.json 2> $O/bench_default.log || { tail -20 $O/bench_default.log; exit 1; }
bline $O/bench_default.json default
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --cpu-sample-stride 0 > $O/bench_prof.json 2> $O/bench_prof.log || { tail -10 $O/bench_prof.log; exit 1; }
cd $R
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/bench_kernel_stats.csv
timeout -k 10 500 python3 tools/shard_cap_timing.py --worlds 2,4 --reps 3 > $O/shard_cap_w24.jsonl 2> $O/shard_cap_w24.log || { tail -20 $O/shard_cap_w24.log; exit 1; }
grep -E "^W=|cap_local parts|restricted" $O/shard_cap_w24.log
timeout -k 10 300 python3 tools/shard_timing.py --reads 1000000 --lmax 16 --seed 11 --worlds 1,2,4,8 > $O/shard_cfg4.jsonl 2> $O/shard_cfg4.log || { tail -20 $O/shard_cfg4.log; exit 1; }
grep -E "^W=" $O/shard_cfg4.log
echo done
