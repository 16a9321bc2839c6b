#!/bin/bash
# Round-4: smoke, the GPU suite, the default bench and the 6-wave fused pair-stage variant, the cfg5
# cap replay's closure variants (component diagnostics on), the sharded cap timing model at cfg5 W=8.
set -o pipefail
TAG=${1:-r4e}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
( while sleep 50; do echo "tick $(date +%T)"; done ) &
TICK=$!
trap "kill $TICK" EXIT
bline() { python3 -c "import json; d=json.load(open('$1')); r=d['roofline']; print('$2', 'ms/step %.4f' % d['ms_per_step'], r['kernel'], '%.4f' % r['kernel_ms'], [(x['kernel'], round(x['kernel_ms'],4)) for x in d.get('roofline_other_kernels', [])], {k: round(v, 3) for k, v in r['phase_ms_last_step'].items()})"; }
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 --cpu-sample-stride 0 > $O/bench_default.json 2> $O/bench_default.log || { tail -20 $O/bench_default.log; exit 1; }
bline $O/bench_default.json default
FSLR_LIB=$R/fslr_amd/libfslr_hip_lds6.so FSLR_ALLOW_STALE=1 FSLR_PAIR_STAGE=fused timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 --cpu-sample-stride 0 > $O/bench_fused_lds6.json 2> $O/bench_fused_lds6.log || { tail -20 $O/bench_fused_lds6.log; exit 1; }
bline $O/bench_fused_lds6.json fused_lds6
FSLR_DEBUG_CAP=1 timeout -k 10 300 python3 tools/cfg5_cap.py --reps 3 > $O/cfg5_cap_frontier.json 2> $O/cfg5_cap_frontier.log || { tail -20 $O/cfg5_cap_frontier.log; exit 1; }
grep "fslr: cap" $O/cfg5_cap_frontier.log | tail -1
python3 -c "import json; d=json.load(open('$O/cfg5_cap_frontier.json')); print('cfg5 frontier+components rep_ms', d['rep_ms'], d.get('full_equal'))"
FSLR_CAP_CLOSURE=rounds timeout -k 10 300 python3 tools/cfg5_cap.py --reps 3 > $O/cfg5_cap_rounds.json 2> $O/cfg5_cap_rounds.log || { tail -20 $O/cfg5_cap_rounds.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/cfg5_cap_rounds.json')); print('cfg5 rounds+components rep_ms', d['rep_ms'], d.get('full_equal'))"
timeout -k 10 400 python3 tools/shard_cap_timing.py --worlds 8 --reps 3 > $O/shard_cap_w8.jsonl 2> $O/shard_cap_w8.log || { tail -20 $O/shard_cap_w8.log; exit 1; }
tail -3 $O/shard_cap_w8.log
echo done
