#!/bin/bash
# A/B of the cfg5 one-GPU cap replay between library variants (fslr_amd/libfslr_hip_<v>.so, main = the
# default library): per-stage times (FSLR_DEBUG_CAP) of tools/cfg5_cap.py.  Usage: tools/cap_ab.sh TAG v1 v2 ...
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
for v in "$@"; do
  lib=$R/fslr_amd/libfslr_hip_$v.so
  [ "$v" = main ] && lib=$R/fslr_amd/libfslr_hip.so
  FSLR_DEBUG_CAP=1 FSLR_LIB=$lib FSLR_ALLOW_STALE=1 timeout -k 10 400 python3 -u tools/cfg5_cap.py --reps 3 \
      > $O/capab_$v.json 2> $O/capab_$v.log || { echo "cap_ab $v failed"; tail -20 $O/capab_$v.log; exit 1; }
  echo "== $v"; grep "cap stage" $O/capab_$v.log | sort | awk '{k=$4; for (i = 5; i <= NF - 2; ++i) k = k " " $i; s[k]+=$(NF-1); c[k]++} END {for (k in s) printf "  %-18s %8.3f ms\n", k, s[k]/c[k]}'
done
