#!/bin/bash
# Round 6: the replay with its loads ahead (product library) against the round-5 replay (libfslr_hip_rv1.so,
# -DFSLR_CAP_REPLAY_V1), by rocprof kernel times of the cfg5 one-GPU cap (no FSLR_DEBUG_CAP: its stage clock
# also holds host-side statistics).  Usage: gpurun -- bash tools/r6_replay_ab.sh TAG
set -o pipefail
TAG=${1:-r6za}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
( while sleep 50; do echo "tick $(date +%T)"; done ) &
TICK=$!
trap "kill $TICK" EXIT
timeout -k 10 600 python -u -m pytest tests/ --maxfail=1 -q --timeout 300 --timeout-method thread -m gpu -k "cap or config5 or dist or multi or shard or long" > $O/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for v in main rv1; do
  lib=$R/fslr_amd/libfslr_hip_$v.so
  [ "$v" = main ] && lib=$R/fslr_amd/libfslr_hip.so
  ( cd /tmp && export TMPDIR=/tmp FSLR_LIB=$lib FSLR_ALLOW_STALE=1 && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run --output-format csv \
      -- python3 $R/tools/cfg5_cap.py --reps 3 > $O/cfg5_cap_$v.json 2> $O/cfg5_cap_$v.log ) || { echo "$v failed"; tail -20 $O/cfg5_cap_$v.log; exit 1; }
  f=$(find $O/prof_$v -name 'run_kernel_stats.csv' | head -1); cp $f $O/kstats_$v.csv; rm -rf $O/prof_$v
  python3 - $O/kstats_$v.csv $v <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'k_cap_replay' in r['Name'] or 'k_cap_sched' in r['Name']:
        print(sys.argv[2], r['Name'].split('(')[0].split('::')[-1], 'mean %.1f us x%s' % (float(r['AverageNs']) / 1000, r['Calls']))
PY
  tail -1 $O/cfg5_cap_$v.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v rep_ms', d['rep_ms'], 'equal', d.get('full_equal'))"
done
echo done
