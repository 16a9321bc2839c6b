#!/bin/bash
# Rehearse the N-rank bench on ONE GPU (gloo transport, all ranks on device 0), with label check.
# Usage (GPU box, repo root): bash tools/rehearse_multi.sh [N]
N=${1:-2}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
FSLR_BENCH_BACKEND=gloo FSLR_BENCH_DEVICE=0 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node $N --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus $N --steps 5 --warmup 2 \
  --cpu-sample-stride 0 --verify > gpurun_out/rehearse_$N.json 2> gpurun_out/rehearse_$N.log
rc=$?
tail -3 gpurun_out/rehearse_$N.log
cat gpurun_out/rehearse_$N.json
exit $rc
