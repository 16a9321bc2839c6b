#!/bin/bash
# quick tests (sweep / cap / dist / long), bench + kernel table, then the cfg5 cap replay timing
# with its full-graph digests (tools/cfg5_cap.py) and kernel stats
set -o pipefail
TAG=${1:-r3d}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/quick_gpu.sh $TAG "(sweep or cap or dist or long) and not slow" || exit 1
bash tools/gpu_cap_prof.sh ${TAG}_cap || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/${TAG}_cap/cfg5_cap.json').read().strip().splitlines()[-1]); print('cfg5 rep_ms', d['rep_ms'], 'query_ms', d['query_ms'], 'full_equal', d.get('full_equal'))"
