#!/bin/bash
# one pytest run on the GPU box: bash tools/gpu_tests.sh TAG <pytest args...>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-t}
shift
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu "$@" > $O/pytest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/pytest.log | tail -60
exit $rc
