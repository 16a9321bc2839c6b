#!/bin/bash
# r3d (quick tests, bench, cfg5 cap replay) + the cfg4 shard timing model (with repeat steps)
set -o pipefail
TAG=${1:-r3f}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/gpu_r3d.sh $TAG || exit 1
O=$R/gpurun_out/${TAG}_shard
mkdir -p $O
timeout -k 10 400 python3 tools/shard_timing.py --reads 1000000 --lmax 16 --seed 11 > $O/shard_cfg4.json 2> $O/shard_cfg4.log \
    || { tail -5 $O/shard_cfg4.log; exit 1; }
grep "W=" $O/shard_cfg4.log
