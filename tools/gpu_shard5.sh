#!/bin/bash
# cfg5 per-rank timing model (10M x 1-64 Zipf, seed 13), with repeat steps
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-shard5}
mkdir -p $O
cd $R
( while sleep 50; do echo "tick $(date +%T)"; done ) &
TICK=$!
trap "kill $TICK" EXIT
timeout -k 10 900 python3 tools/shard_timing.py --reads 10000000 --lmax 64 --dist zipf --seed 13 --reps 3 \
    > $O/shard_cfg5.json 2> $O/shard_cfg5.log || { tail -5 $O/shard_cfg5.log; exit 1; }
grep "W=" $O/shard_cfg5.log
