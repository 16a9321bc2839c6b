#!/bin/bash
# One GPU call: the whole GPU suite + smoke on the tree's library, then per library variant
# (fslr_amd/libfslr_hip_<v>.so, tools/build_variant.sh) the sweep parity subset, a bench line and a
# rocprofv3 kernel table.  Usage: gpurun -- bash tools/gpu_ab.sh TAG [full|none] v1 v2 ...
set -o pipefail
TAG=$1; SUITE=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
( while sleep 50; do echo "tick $(date +%T)"; done ) &
TICK=$!
trap "kill $TICK" EXIT
if [ "$SUITE" = full ]; then
  timeout -k 10 900 python -u -m pytest tests/ -x -q --timeout 300 --timeout-method thread -m gpu > $O/pytest_gpu.log 2>&1 \
      || { echo "gpu tests failed"; tail -40 $O/pytest_gpu.log; exit 1; }
  tail -2 $O/pytest_gpu.log
  timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
fi
for v in "$@"; do
  lib=$R/fslr_amd/libfslr_hip_$v.so
  [ "$v" = main ] && lib=$R/fslr_amd/libfslr_hip.so
  export FSLR_LIB=$lib FSLR_ALLOW_STALE=1
  timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -m gpu \
      -k "sweep and (synthetic or dense or locus or gate or kat or zero or capbind)" > $O/pytest_$v.log 2>&1 \
      || { echo "$v: parity failed"; tail -30 $O/pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/pytest_$v.log)"
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --cpu-sample-stride 0 > $O/bench_$v.json 2> $O/bench_$v.log \
      || { tail -20 $O/bench_$v.log; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$v.json')); r=d['roofline']; print('$v', 'ms/step %.4f' % d['ms_per_step'], r['kernel'], 'kernel_ms %.4f' % r['kernel_ms'], r.get('phase_ms_last_step'), [(k['kernel'], round(k['kernel_ms'],4)) for k in r.get('roofline_other_kernels', [])])"
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run --output-format csv \
      -- python3 $R/bench.py --steps 10 --warmup 2 --cpu-sample-stride 0 > $O/prof_$v.log 2>&1 ) || { echo "$v: rocprof failed"; exit 1; }
  f=$(find $O/prof_$v -name 'run_kernel_stats.csv' | head -1); cp $f $O/kstats_$v.csv
  python3 - $O/kstats_$v.csv <<'PY'
import csv, re, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:10]:
    n = re.sub(r'^void ', '', r['Name'].replace('(anonymous namespace)::', '')); i = n.find('('); n = n[:i] if i > 0 else n
    print(f"   {float(r['AverageNs'])/1000:9.1f} us  x{r['Calls']:>4}  {n[:80]}")
PY
done
echo done
