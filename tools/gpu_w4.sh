#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest -q --maxfail=10 --timeout 120 --timeout-method thread tests/test_gemm_persistent_gpu.py tests/test_kernels_gpu.py -k "gemm or conv" > $OUT/t_w4.log 2>&1
rc=$?; tail -4 $OUT/t_w4.log
if [ $rc -gt 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 400 python tools/gemm_bench.py --sweep > $OUT/gemm_sweep_w4.log 2>&1 || { echo "bench rc=$?"; tail -3 $OUT/gemm_sweep_w4.log; exit 1; }
cat $OUT/gemm_sweep_w4.log
