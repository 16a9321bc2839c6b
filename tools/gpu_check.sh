#!/bin/bash
# One GPU call on the tree's sources (gpurun -- bash tools/gpu_check.sh TAG [STEPS]): STEPS is a comma list
# of tests (the whole GPU suite), smoke, bench (the default bench line), prof (rocprofv3 kernel table of a
# short bench), cli10m (the 10M-read cfg5 CLI, native I/O, stage table), pmc (HBM traffic passes).
# Every step runs under its own time limit; the first failure ends the call.
set -o pipefail
TAG=${1:-chk}
STEPS=${2:-tests,smoke,bench,prof}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
( while sleep 50; do echo "tick $(date +%T)"; done ) &
TICK=$!
trap "kill $TICK" EXIT
has() { [[ ",$STEPS," == *",$1,"* ]]; }
if has tests; then
  timeout -k 10 900 python -u -m pytest tests/ --maxfail=5 -q --timeout 300 --timeout-method thread -m gpu > $O/pytest_gpu.log 2>&1 \
      || { echo "gpu tests failed"; tail -40 $O/pytest_gpu.log; exit 1; }
  tail -2 $O/pytest_gpu.log
fi
if has smoke; then
  timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
fi
if has bench; then
  timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.log || { tail -20 $O/bench.log; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench.json')); r=d['roofline']; print('value %.4e ms/step %.4f cold %s kernel %s %.4f ms frac %.3f' % (d['value'], d['ms_per_step'], d['config'].get('cold_step_ms'), r['kernel'], r['kernel_ms'], r['frac']), r.get('phase_ms_last_step'))"
fi
if has prof; then
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv \
      -- python3 $R/bench.py --steps 10 --warmup 2 --cpu-sample-stride 0 > $O/prof.log 2>&1 ) || { echo "rocprof failed"; tail -5 $O/prof.log; exit 1; }
  f=$(find $O/prof -name 'run_kernel_stats.csv' | head -1); cp $f $O/kernel_stats.csv
  python3 - $O/kernel_stats.csv <<'PY'
import csv, re, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:14]:
    n = re.sub(r'^void ', '', r['Name'].replace('(anonymous namespace)::', '')); i = n.find('('); n = n[:i] if i > 0 else n
    print(f"   {float(r['AverageNs'])/1000:9.1f} us  x{r['Calls']:>4}  {n[:80]}")
PY
fi
if has cli10m; then
  export TMPDIR=${TMPDIR:-/tmp}
  { df -T $TMPDIR | tail -1; python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)))"; } > $O/cli_env.txt 2>&1 || true
  timeout -k 10 600 python3 -u tools/cli_io_timing.py 10000000 64 13 $O/cli_10m.json zipf --native-io > $O/cli_10m.log 2>&1 \
      || { echo "cli10m failed"; tail -20 $O/cli_10m.log; exit 1; }
  tail -3 $O/cli_10m.log
fi
if has hist; then
  # the measurement build is made here on demand (it does not travel with the tree: .gpurunignore)
  timeout -k 10 600 bash tools/build_variant.sh hist -DFSLR_PAIRS_HIST > $O/build_hist.log 2>&1 || { tail -20 $O/build_hist.log; exit 1; }
  FSLR_LIB=$R/fslr_amd/libfslr_hip_hist.so FSLR_ALLOW_STALE=1 timeout -k 10 300 python3 tools/pairs_hist.py $O/pairs_group_hist.json \
      > $O/hist.log 2>&1 || { echo "hist failed"; tail -20 $O/hist.log; exit 1; }
  tail -30 $O/hist.log
  FSLR_LIB=$R/fslr_amd/libfslr_hip_hist.so FSLR_ALLOW_STALE=1 timeout -k 10 500 python3 tools/pairs_hist.py $O/pairs_group_hist_cfg5.json \
      --cfg5 > $O/hist5.log 2>&1 || { echo "hist cfg5 failed"; tail -20 $O/hist5.log; exit 1; }
  tail -30 $O/hist5.log
fi
if has shard; then
  # the per-rank model at 1M reads: both splits, uniform and one chromosome holding ~55 %
  for cfg in "chrom 0" "position 0" "chrom 1.2" "position 1.2"; do
    set -- $cfg
    timeout -k 10 600 python3 -u tools/shard_timing.py --reads 1000000 --lmax 16 --seed 1 --worlds 1,2,4,8 --reps 5 \
        --split $1 --chrom0-weight $2 > $O/shard_$1_$2.jsonl 2> $O/shard_$1_$2.log \
        || { echo "shard $1 $2 failed"; tail -20 $O/shard_$1_$2.log; exit 1; }
    grep "W=8" $O/shard_$1_$2.log || true
  done
fi
if has cfg5; then
  # cfg5 on one GPU under rocprof: the sweep query + the cap replay, checked against the oracle's digests
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/cfg5prof -o run --output-format csv \
      -- python3 $R/tools/cfg5_cap.py --reps 3 > $O/cfg5_cap.json 2> $O/cfg5_cap.log ) || { echo "cfg5 failed"; tail -20 $O/cfg5_cap.log; exit 1; }
  f=$(find $O/cfg5prof -name 'run_kernel_stats.csv' | head -1); cp $f $O/cfg5_kernel_stats.csv
  tail -3 $O/cfg5_cap.log
  python3 - $O/cfg5_kernel_stats.csv <<'PY'
import csv, re, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:12]:
    n = re.sub(r'^void ', '', r['Name'].replace('(anonymous namespace)::', '')); i = n.find('('); n = n[:i] if i > 0 else n
    print(f"   {float(r['AverageNs'])/1000:9.1f} us  x{r['Calls']:>4}  {n[:80]}")
PY
fi
if has rehearse; then
  # the N-rank bench on this one GPU (gloo between ranks, label check)
  for n in 2 4; do
    bash tools/rehearse_multi.sh $n > $O/rehearse_$n.out 2>&1 || { echo "rehearse $n failed"; tail -20 $O/rehearse_$n.out; exit 1; }
    cp gpurun_out/rehearse_$n.json gpurun_out/rehearse_$n.log $O/ 2>/dev/null || true
    tail -1 $O/rehearse_$n.out
  done
fi
if has shardprof; then
  # kernel trace of the W = 8 per-rank model (chromosome split): where a rank's repeat step goes
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/shardprof -o run --output-format csv \
      -- python3 $R/tools/shard_timing.py --reads 1000000 --lmax 16 --seed 1 --worlds 8 --reps 3 > $O/shardprof.log 2>&1 ) \
      || { echo "shardprof failed"; tail -5 $O/shardprof.log; exit 1; }
  f=$(find $O/shardprof -name 'run_kernel_stats.csv' | head -1); cp $f $O/shardprof_kernel_stats.csv
  f=$(find $O/shardprof -name 'run_kernel_trace.csv' | head -1); cp $f $O/shardprof_kernel_trace.csv
fi
if has capmodel; then
  # the sharded cap at cfg5: the per-rank model at W = 8
  timeout -k 10 600 python3 -u tools/shard_cap_timing.py --worlds 8 --reps 3 > $O/capmodel.jsonl 2> $O/capmodel.log \
      || { echo "capmodel failed"; tail -20 $O/capmodel.log; exit 1; }
  tail -3 $O/capmodel.log
fi
if has capshard; then
  # the sharded cap at cfg5, W = 8 ranks on this GPU: per-stage host times (FSLR_DEBUG_CAP), then a kernel trace
  FSLR_DEBUG_CAP=1 timeout -k 10 600 python3 -u tools/shard_cap_timing.py --worlds 8 --reps 1 > $O/capshard_dbg.jsonl 2> $O/capshard_dbg.log \
      || { echo "capshard dbg failed"; tail -20 $O/capshard_dbg.log; exit 1; }
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/capprof -o run --output-format csv \
      -- python3 $R/tools/shard_cap_timing.py --worlds 8 --reps 2 > $O/capshard.jsonl 2> $O/capshard.log ) \
      || { echo "capshard prof failed"; tail -5 $O/capshard.log; exit 1; }
  f=$(find $O/capprof -name 'run_kernel_stats.csv' | head -1); cp $f $O/capshard_kernel_stats.csv
  f=$(find $O/capprof -name 'run_kernel_trace.csv' | head -1); cp $f $O/capshard_kernel_trace.csv
  rm -rf $O/capprof
  tail -3 $O/capshard.log
fi
if has sclock; then
  timeout -k 10 600 bash tools/build_variant.sh sclock -DFSLR_SWEEP_CLOCK > $O/build_sclock.log 2>&1 || { tail -20 $O/build_sclock.log; exit 1; }
  FSLR_LIB=$R/fslr_amd/libfslr_hip_sclock.so FSLR_ALLOW_STALE=1 timeout -k 10 300 python3 tools/sweep_clock.py $O/sweep_clock.json \
      > $O/sclock.log 2>&1 || { echo "sclock failed"; tail -20 $O/sclock.log; exit 1; }
  tail -12 $O/sclock.log
fi
if has bounds; then
  # the whole GPU suite on the bounds-checked build (FSLR_DEBUG_BOUNDS device asserts, kernels.hpp)
  make -s -C fslr_amd/csrc -j16 bounds > $O/build_bounds.log 2>&1 || { tail -20 $O/build_bounds.log; exit 1; }
  FSLR_LIB=$R/fslr_amd/libfslr_hip_bounds.so timeout -k 10 1000 python -u -m pytest tests/ --maxfail=1 -q --timeout 300 \
      --timeout-method thread -m gpu > $O/pytest_bounds.log 2>&1 || { echo "bounds tests failed"; tail -40 $O/pytest_bounds.log; exit 1; }
  tail -2 $O/pytest_bounds.log
fi
if has rccl; then
  # the product's multi-GPU step over RCCL, two ranks sharing this GPU (tools/rccl_one_gpu.py)
  timeout -k 10 300 python3 -u tools/rccl_one_gpu.py $O/rccl_one_gpu.json > $O/rccl.log 2>&1 || { echo "rccl run failed"; tail -20 $O/rccl.log; }
  tail -2 $O/rccl.log
fi
if has pmc; then
  OUT=gpurun_out/$TAG/pmc timeout -k 10 900 bash tools/pmc.sh > $O/pmc.log 2>&1 || { echo "pmc failed"; tail -20 $O/pmc.log; exit 1; }
  tail -5 $O/pmc.log
fi
echo done
