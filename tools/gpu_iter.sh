#!/bin/bash
# Quick GEMM iteration pass: bitwise schedule tests + kernel tests, ablations, per-GEMM step profile.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest -q --maxfail=10 --timeout 120 --timeout-method thread tests/test_gemm_persistent_gpu.py tests/test_kernels_gpu.py > $OUT/t_iter.log 2>&1
rc=$?; tail -4 $OUT/t_iter.log
if [ $rc -gt 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
for c in ${CASES:-qkv_fwd:5 fc2_fwd:5 l1c3_fwd:5}; do
  case_=${c%:*}; tile=${c#*:}
  for d in 0 1; do
    echo -n "dbg=$d "; DFU_GEMM_DEBUG=$d timeout -k 10 60 python tools/gemm_one.py $case_ --tile $tile --iters 30 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
timeout -k 10 300 python tools/gemm_step_profile.py > $OUT/gemm_step_${TAG:-b}.log 2>&1 || { echo "profile rc=$?"; exit 1; }
head -${HEADN:-30} $OUT/gemm_step_${TAG:-b}.log
