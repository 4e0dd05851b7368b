#!/bin/bash
# round 4: stem split pair (tests + bench) and the static-priority GEMM A/B (libdfu_prio.so)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_precision_gpu.py "tests/test_kernels_gpu.py::test_pooling_and_layout" -m gpu -v -x --timeout 200 --timeout-method thread > $OUT/r17_tests.log 2>&1 || { echo "tests rc=$?"; tail -40 $OUT/r17_tests.log; exit 1; }
tail -2 $OUT/r17_tests.log
timeout -k 10 300 python -u -m pytest tests/test_model_parity_gpu.py -m gpu -x -q --timeout 250 --timeout-method thread -k "parity_mode or bf16x3" > $OUT/r17_parity.log 2>&1 || { echo "parity rc=$?"; tail -30 $OUT/r17_parity.log; exit 1; }
tail -2 $OUT/r17_parity.log
AB="DFU_NONE=0 DFU_HIP_LIB=dfu-multimodal_amd/dfu_hip/libdfu_prio.so" REPS=3 STEPS=30 EXTRA="--no-alt-precision --no-parity" bash tools/gpu_ab.sh
