#!/bin/bash
# Round-4 final check on the committed sources: smoke, the GPU suite, the default bench, the CLI at 10M
# reads x 1-64 Zipf (native I/O).
set -o pipefail
TAG=${1:-r4o}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
( while sleep 50; do echo "tick $(date +%T)"; done ) &
TICK=$!
trap "kill $TICK" EXIT
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python3 bench.py > $O/bench_default.json 2> $O/bench_default.log || { tail -20 $O/bench_default.log; exit 1; }
cut -c1-700 $O/bench_default.json
export TMPDIR=/tmp
timeout -k 10 600 python3 tools/cli_io_timing.py 10000000 64 13 $O/cli_10m.json zipf --native-io > $O/cli_10m.log 2>&1 || { tail -20 $O/cli_10m.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/cli_10m.json')); print({k: v for k, v in d.items() if k not in ('extra_args',)})"
echo done
