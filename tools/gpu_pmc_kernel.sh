#!/bin/bash
# PMC passes for one kernel (regex) on a short bench: bash tools/gpu_pmc_kernel.sh TAG REGEX
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/$1/pmc REGEX=$2 bash $R/tools/pmc_kernels.sh > $R/gpurun_out/$1/pmc_summary.txt 2>&1
cat $R/gpurun_out/$1/pmc_summary.txt
