#!/bin/bash
# Final-tree pass: GPU suite, a same-box A/B of the schedule default against the previous one,
# then the round's measurement pass (tools/gpu_round.sh <tag>).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; OUT=$R/gpurun_out; TAG=${1:-r26}; mkdir -p $OUT; cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests_$TAG.txt 2>&1 || { echo "suite rc=$?"; tail -30 $OUT/gpu_tests_$TAG.txt; exit 1; }
tail -1 $OUT/gpu_tests_$TAG.txt
bash tools/gpu_ab_env.sh pfin 2 "X=0" "DFU_GEMM_PERSISTENT=1" || exit 1
bash tools/gpu_round.sh $TAG
