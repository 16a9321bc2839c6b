#!/bin/bash
# round-end measurement: parity subset + bench + kernel stats, then the PMC passes of both sweep kernels
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-final}
cd $R
bash tools/gpu_iter3.sh $TAG "sweep or dense or capbind" || exit 1
OUT=gpurun_out/$TAG/pmc bash tools/pmc.sh > gpurun_out/$TAG/pmc.log 2>&1 || { tail -20 gpurun_out/$TAG/pmc.log; exit 1; }
tail -2 gpurun_out/$TAG/pmc.log
python3 -c "
import json; d=json.load(open('gpurun_out/$TAG/pmc/traffic.json'))
for k, v in d.items(): print(k, 'hbm MB/launch %.1f' % (v['hbm_bytes_per_launch'] / 1e6), 'L2 hit %.2f' % v.get('l2_hit_rate', -1))"
