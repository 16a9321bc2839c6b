#!/bin/bash
# PMC passes for the dominant kernel (separate rocprofv3 runs, --pmc only with --kernel-trace-free collection).
# Usage (GPU box, repo root): OUT=gpurun_out/pmc [ENGINE=sweep|walk] tools/pmc.sh [bench args]
set -e
OUT=${OUT:-gpurun_out/pmc}
ENGINE=${ENGINE:-sweep}
if [ "$ENGINE" = walk ]; then KREGEX="query_kernel"; KNAMES="query_kernel<0, false>"; else KREGEX="k_sweep<2>|k_sweep_pairs"; KNAMES="k_sweep<2>;k_sweep_pairs"; fi
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $ROOT/$OUT
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-include-regex "$KREGEX" -d $ROOT/$OUT/p$i -o pmc \
      --output-format csv -- python3 $ROOT/bench.py --steps 2 --warmup 1 --cpu-sample-stride 0 --engine $ENGINE "$@" \
      > $ROOT/$OUT/p$i.log 2>&1
done
cd $ROOT
H=$(python3 -c "import bench; print(bench.kernel_source_hash('$ENGINE'))")
rm -f $ROOT/$OUT/traffic.json
IFS=';' read -ra KS <<< "$KNAMES"
for K in "${KS[@]}"; do
  python3 tools/pmc_traffic.py $ROOT/$OUT --kernel "$K" --source-hash $H --merge-into $ROOT/$OUT/traffic.json > /dev/null \
    || echo "no rows for $K (not launched by this configuration)"
done
echo "traffic summary: $OUT/traffic.json (source $H; kernels: $KNAMES)"
