#!/bin/bash
# r3d (quick tests, bench, cfg5 cap replay) + pair-kernel ablation variants' kernel times
set -o pipefail
TAG=${1:-r3e}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/gpu_r3d.sh $TAG || exit 1
bash tools/abl_runs.sh ${TAG}_abl main abl1 abl2 abl4 abl5
