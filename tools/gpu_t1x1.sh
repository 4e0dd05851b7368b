#!/bin/bash
# 1x1 transposed-weight dgrads: per-shape timing, GPU tests, same-box A/B (fusion, RGB) with the
# DSTATS epilogue toggle beside it.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 120 python tools/t1x1_time.py > $OUT/t1x1.log 2>&1 || { echo "t1x1 rc=$?"; tail -30 $OUT/t1x1.log; exit 1; }
cat $OUT/t1x1.log | grep -v amdgpu.ids
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_nn_standalone_gpu.py tests/test_blocks_gpu.py tests/test_kernels_gpu.py -m gpu > $OUT/pytest_t1x1.log 2>&1 || { echo "pytest rc=$?"; tail -40 $OUT/pytest_t1x1.log; exit 1; }
tail -2 $OUT/pytest_t1x1.log
AB="DFU_BASE=1 DFU_DGRAD_T1X1_MAXC=0 DFU_FUSE_BN_DSTATS=1" CONFIG=rgb REPS=2 bash tools/gpu_ab.sh || exit 1
AB="DFU_BASE=1 DFU_DGRAD_T1X1_MAXC=0 DFU_FUSE_BN_DSTATS=1" CONFIG=fusion REPS=2 bash tools/gpu_ab.sh || exit 1
