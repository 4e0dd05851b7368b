#!/bin/bash
# A/B of an experiment build (DFU_HIP_LIB=<lib>): GPU tests of the GEMM kernels on it, then the
# step alternating with the product library.  bash tools/gpu_libab.sh <tag> <lib> <rounds> [tests]
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; OUT=$R/gpurun_out; TAG=$1; LIB=$R/$2; N=${3:-3}; mkdir -p $OUT
T=${4:-"tests/test_kernels_gpu.py tests/test_precision_gpu.py"}
DFU_HIP_LIB=$LIB timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread $T > $OUT/t_$TAG.log 2>&1 || { echo "tests rc=$?"; tail -30 $OUT/t_$TAG.log; exit 1; }
tail -1 $OUT/t_$TAG.log
bash tools/gpu_ab_env.sh $TAG $N "X=0" "DFU_HIP_LIB=$LIB"
