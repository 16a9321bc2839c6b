#!/bin/bash
# PMC traffic for the current pair kernel -> profiles/pmc_traffic_latest.json, then the default bench
# (which reads it when the source hash matches).  GPU box, repo root.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=gpurun_out/pmc_latest bash tools/pmc.sh
cd $R
cp gpurun_out/pmc_latest/traffic.json profiles/pmc_traffic_latest.json   # (copy it locally too: only gpurun_out/ returns)
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.log
cat gpurun_out/bench_default.json
