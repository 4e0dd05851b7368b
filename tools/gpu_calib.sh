#!/bin/bash
# Calibration pass (via gpurun): hipBLASLt vs the template on the ViT shapes, then the compile-time
# ablations of the persistent phased GEMM (tools/build_ablate.sh libraries) on a few shapes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 240 python3 tools/blas_compare.py > $OUT/blas_compare.txt 2>&1 || { echo "blas rc=$?"; tail -5 $OUT/blas_compare.txt; exit 1; }
cat $OUT/blas_compare.txt
rm -f $OUT/ablate2.txt
MASKS="${MASKS:-0 1 2 4 5 3}" bash tools/gpu_ablate2.sh ${SHAPES:-fc1_gelu:8 fc2_fwd_resid:8 fc2_wgrad:8 qkv_fwd:8}
