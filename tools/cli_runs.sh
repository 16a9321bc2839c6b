#!/bin/bash
# End-to-end CLI wall times on the GPU box (repo root, via gpurun):
#   bash tools/cli_runs.sh TAG [10m]
# 1M x 1-16 with native and pandas I/O (outputs compared) and with --gpus=2; with "10m" also
# 10M x 1-64 Zipf (cfg5) with native I/O.  A ticker keeps the run visibly alive.
TAG=${1:-cli}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
( while sleep 50; do echo "tick $(date +%T)"; done ) &
TICK=$!
trap "kill $TICK" EXIT
export TMPDIR=${TMPDIR:-/tmp}
timeout -k 10 300 python3 tools/cli_io_timing.py 1000000 16 11 $O/cli_1M.json uniform --native-io,--pandas-io > $O/cli_1M.log 2>&1 || { tail -20 $O/cli_1M.log; exit 1; }
tail -2 $O/cli_1M.log | cut -c1-400
timeout -k 10 200 python3 tools/cli_io_timing.py 1000000 16 11 $O/cli_1M_gpus2.json uniform --native-io,--gpus=2,repeat > $O/cli_1M_gpus2.log 2>&1 || { tail -20 $O/cli_1M_gpus2.log; exit 1; }
tail -1 $O/cli_1M_gpus2.log | cut -c1-400
if [ "$2" = "10m" ]; then
  timeout -k 10 900 python3 tools/cli_io_timing.py 10000000 64 13 $O/cli_10M.json zipf --native-io > $O/cli_10M.log 2>&1 || { tail -20 $O/cli_10M.log; exit 1; }
  tail -1 $O/cli_10M.log | cut -c1-400
fi
