#!/bin/bash
# Round-3 (second session) iteration: sweep / cap / dist GPU tests, bench line, rocprof kernel
# table, and a 2-rank rehearsal of the multi-GPU bench on one GPU (gloo) with the repeat steps
set -o pipefail
TAG=${1:-r3b}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
bash tools/quick_gpu.sh $TAG "(sweep or cap or dist) and not slow" || exit 1
N=2
FSLR_BENCH_BACKEND=gloo FSLR_BENCH_DEVICE=0 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node $N --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus $N --steps 5 --warmup 2 \
  --cpu-sample-stride 0 --verify > $O/rehearse_$N.json 2> $O/rehearse_$N.log || { tail -30 $O/rehearse_$N.log; exit 1; }
python3 -c "import json; d=json.loads(open('$O/rehearse_$N.json').read().strip().splitlines()[-1]); print('rehearse W=2 ms/step %.3f verified %s' % (d['ms_per_step'], d.get('verified_labels_vs_single_context')))"
