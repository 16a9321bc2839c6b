set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/idxv3
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in "" _norec _noload _none; do
  FSLR_LIB=$R/fslr_amd/libfslr_hip$v.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/p$v -o run --output-format csv -- python3 $R/tools/index_timing.py --steps 10 > $O/log$v.txt 2>&1
  f=$(find $O/p$v -name "run_kernel_stats.csv" | head -1)
  echo "== $v"; python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    print('%9.1f us  %s' % (float(r['AverageNs'])/1000, r['Name'][:60]))
" | head -8
done
