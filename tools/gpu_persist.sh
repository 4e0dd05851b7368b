#!/bin/bash
# GPU pass for the persistent GEMM schedule: bitwise + numerics tests, per-GEMM A/B timing, bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest -q --maxfail=20 --timeout 120 --timeout-method thread tests/test_gemm_persistent_gpu.py tests/test_kernels_gpu.py > $OUT/t_persist.log 2>&1
rc=$?
tail -25 $OUT/t_persist.log
if [ $rc -gt 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python tools/gemm_bench.py --ab > $OUT/gemm_ab.log 2>&1 || { echo "gemm_bench rc=$?"; tail -5 $OUT/gemm_ab.log; exit 1; }
cat $OUT/gemm_ab.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench_persist.json 2> $OUT/bench_persist.err || { echo "bench rc=$?"; tail -20 $OUT/bench_persist.err; exit 1; }
cat $OUT/bench_persist.json
