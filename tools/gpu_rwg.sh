#!/bin/bash
# ResNet weight gradients on the wgrad stream (RGB-only): GPU tests touching the ResNet backward,
# then same-box A/B of the RGB-only and fusion steps.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_blocks_gpu.py tests/test_configs_gpu.py tests/test_gradcam_gpu.py tests/test_streams_gpu.py tests/test_model_parity_gpu.py tests/test_dropin_gpu.py -m gpu > $OUT/pytest_rwg.log 2>&1 || { echo "pytest rc=$?"; tail -40 $OUT/pytest_rwg.log; exit 1; }
tail -2 $OUT/pytest_rwg.log
AB="DFU_RESNET_WGRAD_STREAM=1 DFU_RESNET_WGRAD_STREAM=0" CONFIG=rgb REPS=3 bash tools/gpu_ab.sh || exit 1
AB="DFU_RESNET_WGRAD_STREAM=1 DFU_RESNET_WGRAD_STREAM=0" CONFIG=fusion REPS=1 bash tools/gpu_ab.sh || exit 1
