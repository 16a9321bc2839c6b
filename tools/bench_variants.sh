#!/bin/bash
# bench.py (no CPU baseline) for each library variant given: tools/bench_variants.sh TAG v1 v2 ...
# ("" = the default libfslr_hip.so); prints ms/step and pair-kernel ms per variant
set -e
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
for v in "$@"; do
  lib=$R/fslr_amd/libfslr_hip${v:+_$v}.so
  FSLR_LIB=$lib timeout -k 10 200 python $R/bench.py --cpu-sample-stride 0 --steps 20 > $O/bench_${v:-default}.json 2> $O/bench_${v:-default}.log
  python -c "import json,sys; d=json.load(open('$O/bench_${v:-default}.json')); p=d['roofline']['phase_ms_last_step']; print('%-8s ms/step %.4f sweep %.4f sort %.4f pairs %.4f' % ('${v:-default}', d['ms_per_step'], d['roofline']['kernel_ms'], p['sweep_sort_ms'], p['sweep_pairs_ms']))"
done
