#!/bin/bash
# Round 6: k_sweep_pairs chunk size (FSLR_PAIRS_CHUNK 512 = main, 256, 128: libfslr_hip_c256/c128.so) on a
# rank's share (tools/shard_timing.py, position split, W = 8: per-rank evaluate and the repeat step) and on
# one GPU (the bench line).  Usage: gpurun -- bash tools/r6_chunk_ab.sh TAG
set -o pipefail
TAG=${1:-r6n}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
( while sleep 50; do echo "tick $(date +%T)"; done ) &
TICK=$!
trap "kill $TICK" EXIT
for v in main c256 c128; do
  lib=$R/fslr_amd/libfslr_hip_$v.so
  [ "$v" = main ] && lib=$R/fslr_amd/libfslr_hip.so
  export FSLR_LIB=$lib FSLR_ALLOW_STALE=1
  timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -m gpu \
      -k "sweep and (synthetic or dense or locus)" > $O/pytest_$v.log 2>&1 || { echo "$v: parity failed"; tail -30 $O/pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/pytest_$v.log)"
  timeout -k 10 600 python3 -u tools/shard_timing.py --reads 1000000 --lmax 16 --seed 1 --worlds 1,8 --reps 5 \
      --split position > $O/shard_$v.jsonl 2> $O/shard_$v.log || { echo "$v: shard failed"; tail -20 $O/shard_$v.log; exit 1; }
  echo "$v: $(grep 'W=8' $O/shard_$v.log)"
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --cpu-sample-stride 0 > $O/bench_$v.json 2> $O/bench_$v.log \
      || { tail -20 $O/bench_$v.log; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$v.json')); r=d['roofline']; print('$v', 'ms/step %.4f' % d['ms_per_step'], r['kernel'], 'kernel_ms %.4f' % r['kernel_ms'])"
done
echo done
