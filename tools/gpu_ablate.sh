#!/bin/bash
# GEMM ablation timings (DFU_GEMM_DEBUG: 1 no epilogue, 2 no MFMA, 4 no DMA) for single GEMMs.
#   bash tools/gpu_ablate.sh fc1_fwd:13 fc2_fwd:13 ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
for spec in "$@"; do
  case_=${spec%:*}; tile=${spec#*:}
  for dbg in ${DBGS:-0 1 2 4 6 5}; do
    echo -n "dbg $dbg: " >> $OUT/ablate.txt
    DFU_GEMM_DEBUG=$dbg timeout -k 10 60 python3 tools/gemm_one.py $case_ --tile $tile --iters 20 2>/dev/null >> $OUT/ablate.txt || exit 1
  done
done
cat $OUT/ablate.txt
