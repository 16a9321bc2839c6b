#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration on known byte counts (tools/microbench/fetchcal.hip), one rocprofv3
# --pmc pass per counter.  Usage (GPU box, repo root): OUT=gpurun_out/cal bash tools/fetchcal.sh
set -e
OUT=${OUT:-gpurun_out/cal}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $ROOT/$OUT
hipcc -O3 --offload-arch=gfx950 -o $ROOT/$OUT/fetchcal $ROOT/tools/microbench/fetchcal.hip
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 $ROOT/$OUT/fetchcal > $ROOT/$OUT/known.json
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c -d $ROOT/$OUT/$c -o pmc --output-format csv -- $ROOT/$OUT/fetchcal \
      > $ROOT/$OUT/$c.log 2>&1
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/trace -o run --output-format csv -- $ROOT/$OUT/fetchcal \
    > $ROOT/$OUT/trace.log 2>&1
cd $ROOT
python3 tools/fetch_calibration.py $OUT -o $OUT/fetch_calibration.json
