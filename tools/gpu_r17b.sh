#!/bin/bash
# round 4: ReLU bitmasks in the x3 backward -- tests, parity, bench, per-kernel PMC bytes
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 300 python -u -m pytest tests/test_precision_gpu.py tests/test_blocks_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/r17b_tests.log 2>&1 || { echo "tests rc=$?"; tail -40 $OUT/r17b_tests.log; exit 1; }
tail -2 $OUT/r17b_tests.log
timeout -k 10 400 python -u -m pytest tests/test_model_parity_gpu.py tests/test_gradcam_gpu.py -m gpu -x -q -s --timeout 300 --timeout-method thread > $OUT/r17b_parity.log 2>&1 || { echo "parity rc=$?"; tail -30 $OUT/r17b_parity.log; exit 1; }
grep -E "C3 B=64|passed|failed" $OUT/r17b_parity.log | tail -6
REPS=2 AB="DFU_NONE=0 DFU_VIT_WGRAD_SPLIT_DIV=2 DFU_VIT_WGRAD_SPLIT_DIV=3" STEPS=30 EXTRA="--no-alt-precision --no-parity" bash tools/gpu_ab.sh || exit 1
bash tools/gpu_pmc_step.sh pmcpar2 | head -22
