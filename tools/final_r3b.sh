#!/bin/bash
# Round-3 final pass on the box: PMC traffic of both sweep kernels on these sources (into
# profiles/pmc_traffic_latest.json, which the bench reads), then what the driver runs at round end
# (the whole GPU suite, smoke, the default bench line), then the rocprof kernel table of the bench
set -o pipefail
TAG=${1:-final3b}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
( while sleep 50; do echo "tick $(date +%T)"; done ) &
TICK=$!
trap "kill $TICK" EXIT
OUT=gpurun_out/$TAG/pmc bash tools/pmc.sh > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
tail -1 $O/pmc.log
cp $O/pmc/traffic.json profiles/pmc_traffic_latest.json
cp $O/pmc/traffic.json $O/pmc_traffic_latest.json
bash tools/round_end.sh $TAG || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
    python3 $R/bench.py --steps 10 --warmup 3 --cpu-sample-stride 0 > $O/prof_bench.json 2> $O/prof.log || { tail -5 $O/prof.log; exit 1; }
echo final pass done
