#!/bin/bash
# GPU pass: per-GEMM step profile (current plans, A/B schedules), then re-tune the plan table.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 300 python tools/gemm_step_profile.py --ab > $OUT/gemm_step_${1:-a}.log 2>&1 || { echo "profile rc=$?"; tail -5 $OUT/gemm_step_${1:-a}.log; exit 1; }
head -60 $OUT/gemm_step_${1:-a}.log
timeout -k 10 600 python tools/gemm_tune.py --out $OUT/gemm_tuned.inc > $OUT/gemm_tune.log 2>&1 || { echo "tune rc=$?"; tail -5 $OUT/gemm_tune.log; exit 1; }
tail -3 $OUT/gemm_tune.log
