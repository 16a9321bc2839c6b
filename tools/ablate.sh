#!/bin/bash
# Pair-kernel ablation + PMC passes (run on the GPU box from the repo root).
set -e
OUT=${OUT:-gpurun_out/ablate}
mkdir -p $OUT
for m in 0 1 2; do
  FSLR_ABLATE=$m timeout -k 10 300 python bench.py --steps 5 --warmup 1 --cpu-sample-reads 0 > $OUT/bench_mode$m.json 2> $OUT/bench_mode$m.log
done
