#!/bin/bash
# Time library variants with bench.py (GPU box).  Usage: tools/variants.sh name1 name2 ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for v in "$@"; do
  lib=$R/fslr_amd/libfslr_hip_$v.so
  [ "$v" = main ] && lib=$R/fslr_amd/libfslr_hip.so
  FSLR_LIB=$lib timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-sample-reads 0 > gpurun_out/var_$v.json 2> gpurun_out/var_$v.log || exit 1
  python -c "import json; d=json.load(open('gpurun_out/var_$v.json')); print('$v', 'ms/step %.4f' % d['ms_per_step'], 'kernel_ms %.4f' % d['roofline']['kernel_ms'], 'pairs %d' % d['config']['evaluated_pairs_per_step'])"
done
