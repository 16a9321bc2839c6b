#!/bin/bash
# sweep / dist / long GPU tests, bench line, cfg4 shard model
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-gp}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "(sweep or dist or long or parity) and not slow" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --cpu-sample-stride 0 > $O/bench.json 2> $O/bench.log || { tail -20 $O/bench.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); r=d['roofline']; print('value %.4e ms/step %.3f' % (d['value'], d['ms_per_step']), r['phase_ms_last_step'])"
timeout -k 10 400 python3 tools/shard_timing.py --reads 1000000 --lmax 16 --seed 11 > $O/shard_cfg4.json 2> $O/shard_cfg4.log || { tail -5 $O/shard_cfg4.log; exit 1; }
grep "W=" $O/shard_cfg4.log
