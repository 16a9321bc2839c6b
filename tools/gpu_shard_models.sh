#!/bin/bash
# per-rank timing model of the chromosome split: cfg4 (1M x 1-16) and cfg5 (10M x 1-64 Zipf, seed 13)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-shard3}
mkdir -p $O
cd $R
( while sleep 50; do echo "tick $(date +%T)"; done ) &
TICK=$!
trap "kill $TICK" EXIT
timeout -k 10 400 python3 tools/shard_timing.py --reads 1000000 --lmax 16 --seed 11 > $O/shard_cfg4.json 2> $O/shard_cfg4.log \
    || { tail -5 $O/shard_cfg4.log; exit 1; }
tail -2 $O/shard_cfg4.log
timeout -k 10 700 python3 tools/shard_timing.py --reads 10000000 --lmax 64 --dist zipf --seed 13 --reps 3 \
    > $O/shard_cfg5.json 2> $O/shard_cfg5.log || { tail -5 $O/shard_cfg5.log; exit 1; }
tail -2 $O/shard_cfg5.log
