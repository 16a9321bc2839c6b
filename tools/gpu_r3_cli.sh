#!/bin/bash
# round 3: CLI fixtures (columnar + pandas paths, --gpus=2), the large configs, then CLI wall times
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-cli3}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
( while sleep 50; do echo "tick $(date +%T)"; done ) &
TICK=$!
trap "kill $TICK" EXIT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
    -k "cli" > $O/pytest_cli.log 2>&1 || { echo "cli tests failed"; tail -30 $O/pytest_cli.log; exit 1; }
tail -1 $O/pytest_cli.log
if [ "$2" != "nocfg" ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_configs.py \
      > $O/pytest_configs.log 2>&1 || { echo "config tests failed"; tail -30 $O/pytest_configs.log; exit 1; }
  tail -1 $O/pytest_configs.log
fi
[ "$2" = "nocli" ] && exit 0
bash tools/cli_runs.sh $TAG 10m
