#!/bin/bash
# End-of-round GPU pass (repo root): all GPU tests + smoke, PMC traffic of the sweep kernel for the
# committed sources, rocprof kernel trace of the bench, the bench line, cfg5 cap-replay stage timing
# and the cfg4 per-rank shard timing.  Usage: bash tools/final_round.sh TAG
TAG=${1:-final}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
OUT=gpurun_out/$TAG/pmc bash tools/pmc.sh || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --cpu-sample-stride 0 > $O/prof_bench.json 2> $O/prof.log || { tail -20 $O/prof.log; exit 1; }
cd $R
cp $O/pmc/traffic.json profiles/pmc_traffic_latest.json
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.log || { tail -20 $O/bench.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); r=d['roofline']; print('value %.4e ms/step %.3f frac %.3f traffic %s waste %s' % (d['value'], d['ms_per_step'], r['frac'], r['traffic'], r.get('waste_ratio')))"
FSLR_CAP_TIMING=1 timeout -k 10 400 python3 tools/cfg5_check.py --cap --sample 50000 --oracle-npz tests/golden/cfg5/sample50k_capped.npz --steps 2 > $O/cfg5.json 2> $O/cfg5.log || { tail -20 $O/cfg5.log; exit 1; }
grep -E "cap\]|replay|device step|parity|match" $O/cfg5.log | head -20
timeout -k 10 300 python3 tools/shard_timing.py --reads 1000000 --lmax 16 --seed 11 > $O/shard_cfg4.jsonl 2> $O/shard_cfg4.log || { tail -20 $O/shard_cfg4.log; exit 1; }
grep "W=" $O/shard_cfg4.log
