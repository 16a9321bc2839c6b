#!/bin/bash
# cap replay: parity tests (one GPU, split, long reads), then the cfg5 replay profile
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-capit}
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_long.py tests/test_dist.py -x -q --timeout 300 \
    --timeout-method thread -m gpu -k "cap or long or dense" > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/gpu_cap_prof.sh ${1:-capit}
