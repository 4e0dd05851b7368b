#!/bin/bash
# bf16x3 weight-operand cache: GPU tests, then same-box A/B of the bf16x3 fusion step.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_precision_gpu.py tests/test_model_parity_gpu.py tests/test_configs_gpu.py -m gpu > $OUT/pytest_x3c.log 2>&1 || { echo "pytest rc=$?"; tail -40 $OUT/pytest_x3c.log; exit 1; }
tail -2 $OUT/pytest_x3c.log
AB="DFU_X3_WEIGHT_CACHE=1 DFU_X3_WEIGHT_CACHE=0" CONFIG=fusion REPS=3 EXTRA="--precision bf16x3 --no-alt-precision --no-parity" bash tools/gpu_ab.sh || exit 1
