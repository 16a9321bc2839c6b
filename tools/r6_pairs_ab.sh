#!/bin/bash
# Round 6: the bucketed long-run path of k_sweep_pairs against the partition path (libfslr_hip_oldlr.so,
# -DFSLR_PAIRS_NO_BUCKETS): the GPU suite on the product library, then per library the cfg3 bench line and
# rocprof table, and cfg5's sweep query + cap under rocprof.  Usage: gpurun -- bash tools/r6_pairs_ab.sh TAG
set -o pipefail
TAG=${1:-r6h}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
( while sleep 50; do echo "tick $(date +%T)"; done ) &
TICK=$!
trap "kill $TICK" EXIT
timeout -k 10 900 python -u -m pytest tests/ --maxfail=1 -q --timeout 300 --timeout-method thread -m gpu > $O/pytest_gpu.log 2>&1 \
    || { echo "gpu tests failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for v in main oldlr; do
  lib=$R/fslr_amd/libfslr_hip_$v.so
  [ "$v" = main ] && lib=$R/fslr_amd/libfslr_hip.so
  export FSLR_LIB=$lib FSLR_ALLOW_STALE=1
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --cpu-sample-stride 0 > $O/bench_$v.json 2> $O/bench_$v.log \
      || { tail -20 $O/bench_$v.log; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$v.json')); r=d['roofline']; print('$v', 'ms/step %.4f' % d['ms_per_step'], r['kernel'], 'kernel_ms %.4f' % r['kernel_ms'])"
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/cfg5prof_$v -o run --output-format csv \
      -- python3 $R/tools/cfg5_cap.py --reps 2 > $O/cfg5_cap_$v.json 2> $O/cfg5_cap_$v.log ) || { echo "$v cfg5 failed"; tail -20 $O/cfg5_cap_$v.log; exit 1; }
  f=$(find $O/cfg5prof_$v -name 'run_kernel_stats.csv' | head -1); cp $f $O/cfg5_kernel_stats_$v.csv; rm -rf $O/cfg5prof_$v
  tail -2 $O/cfg5_cap_$v.log
  python3 - $O/cfg5_kernel_stats_$v.csv <<'PY'
import csv, re, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:6]:
    n = re.sub(r'^void ', '', r['Name'].replace('(anonymous namespace)::', '')); i = n.find('('); n = n[:i] if i > 0 else n
    print(f"   {float(r['AverageNs'])/1000:9.1f} us  x{r['Calls']:>4}  {n[:80]}")
PY
done
unset FSLR_LIB FSLR_ALLOW_STALE
bash tools/gpu_check.sh $TAG hist
