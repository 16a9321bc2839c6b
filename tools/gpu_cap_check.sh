#!/bin/bash
# cap replay parity tests + cfg5 cap timing (one GPU call)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_dist.py -x -v --timeout 300 --timeout-method thread -m gpu -k "sweep_split or capped_one_gpu" > gpurun_out/r3_t1.log 2>&1 && \
timeout -k 10 600 python -u tools/cfg5_cap.py --reps 3 > gpurun_out/r3_cfg5cap.json 2> gpurun_out/r3_cfg5cap.log
