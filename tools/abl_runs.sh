#!/bin/bash
# Kernel times of library variants (profiling ablations) under rocprofv3 --stats:
#   bash tools/abl_runs.sh TAG main abl1 abl2 ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  lib=$R/fslr_amd/libfslr_hip_$v.so
  [ "$v" = main ] && lib=$R/fslr_amd/libfslr_hip.so
  FSLR_ABLATE=1 FSLR_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$v -o run --output-format csv -- \
      python3 $R/bench.py --steps 10 --warmup 2 --cpu-sample-stride 0 > $O/$v.json 2> $O/$v.log || echo "$v: bench exited non-zero (ablations may overflow buffers after timing)"
  python3 - $O/$v/run_kernel_stats.csv $v <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
want = ('k_sweep_pairs', 'k_sweep<2>', 'k_msd_pass1', 'k_msd_pass2', 'k_chrom_scatter')
import re
def short(n):
    m = re.search(r'(k_\w+(<[^>]*>)?)', n)
    return m.group(1) if m else n[:30]
print(sys.argv[2], ' '.join(f"{short(r['Name'])}={float(r['AverageNs'])/1000:.1f}us" for r in rows
                           if any(w in r['Name'] for w in want)))
PY
done
