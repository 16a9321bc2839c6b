#!/bin/bash
# sweep parity + multi-GPU CLI/pool tests, bench + kernel stats, then the 1M --gpus=2 CLI timing
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-it6}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -m gpu \
    -k "multi_gpu or rank_pool" > $O/pytest_multi.log 2>&1 || { echo "multi tests failed"; tail -30 $O/pytest_multi.log; exit 1; }
tail -1 $O/pytest_multi.log
bash tools/gpu_iter3.sh ${1:-it6} "sweep or dense or capbind" || exit 1
export TMPDIR=${TMPDIR:-/tmp}
timeout -k 10 200 python3 tools/cli_io_timing.py 1000000 16 11 $O/cli_1M_gpus2.json uniform --native-io,--gpus=2,repeat \
    > $O/cli_1M_gpus2.log 2>&1 || { tail -20 $O/cli_1M_gpus2.log; exit 1; }
tail -1 $O/cli_1M_gpus2.log | cut -c1-600
