#!/bin/bash
# Round-4: the frontier rounds' grid (A/B 1024 / 256 / 128 workgroups) on the cfg5 cap replay, the suite.
set -o pipefail
TAG=${1:-r4r}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
( while sleep 50; do echo "tick $(date +%T)"; done ) &
TICK=$!
trap "kill $TICK" EXIT
for g in 1024 256 128; do
  FSLR_CAP_FGRID=$g timeout -k 10 300 python3 tools/cfg5_cap.py --reps 5 > $O/cfg5_cap_g$g.json 2> $O/cfg5_cap_g$g.log || { tail -20 $O/cfg5_cap_g$g.log; exit 1; }
  python3 -c "import json; d=json.load(open('$O/cfg5_cap_g$g.json')); print('grid $g rep_ms', d['rep_ms'], d.get('full_equal'))"
done
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
echo done
