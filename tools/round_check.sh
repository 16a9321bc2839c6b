#!/bin/bash
# Full GPU check (repo root, via gpurun): all GPU tests, default bench line, shard timing at cfg4
# (1M x 1-16) and cfg5 (10M x 1-64 Zipf).  Usage: bash tools/round_check.sh TAG [skip-cfg5]
TAG=${1:-rc}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 > $O/bench.json 2> $O/bench.log || { tail -20 $O/bench.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print('value %.4e ms/step %.3f frac %.3f' % (d['value'], d['ms_per_step'], d['roofline']['frac']))"
timeout -k 10 300 python3 tools/shard_timing.py --reads 1000000 --lmax 16 --seed 11 > $O/shard_cfg4.jsonl 2> $O/shard_cfg4.log || { tail -20 $O/shard_cfg4.log; exit 1; }
grep "W=" $O/shard_cfg4.log
if [ "$2" != "skip-cfg5" ]; then
  timeout -k 10 400 python3 tools/shard_timing.py --reads 10000000 --lmax 64 --dist zipf --seed 13 --reps 3 > $O/shard_cfg5.jsonl 2> $O/shard_cfg5.log || { tail -20 $O/shard_cfg5.log; exit 1; }
  grep "W=" $O/shard_cfg5.log
fi
