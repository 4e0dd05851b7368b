#!/bin/bash
# Early AdamW of the main stream's deep-stage block: GPU tests, then same-box A/B (fusion, RGB).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_optim_gpu.py tests/test_dropin_gpu.py tests/test_streams_gpu.py tests/test_loop_gpu.py tests/test_golden_gpu.py -m gpu > $OUT/pytest_eam.log 2>&1 || { echo "pytest rc=$?"; tail -40 $OUT/pytest_eam.log; exit 1; }
tail -2 $OUT/pytest_eam.log
AB="DFU_EARLY_ADAMW_MAIN=1 DFU_EARLY_ADAMW_MAIN=0" CONFIG=fusion REPS=3 bash tools/gpu_ab.sh || exit 1
AB="DFU_EARLY_ADAMW_MAIN=1 DFU_EARLY_ADAMW_MAIN=0" CONFIG=rgb REPS=2 bash tools/gpu_ab.sh || exit 1
