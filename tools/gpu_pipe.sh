#!/bin/bash
# GPU pass for the pipelined K-loop tiles: GEMM correctness over every tile, then a full tune
# of the step's GEMMs over tiles 1..12 (table + per-shape timing dump into gpurun_out/).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_gemm_persistent_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_pipe.log 2>&1 || { echo "pytest rc=$?"; tail -30 $OUT/pytest_pipe.log; exit 1; }
tail -2 $OUT/pytest_pipe.log
timeout -k 10 600 python -u tools/gemm_tune.py --iters 10 --tiles ${TILES:-1-12} --out $OUT/tuned_pipe.inc --dump $OUT/tune_pipe.json > $OUT/tune_pipe.log 2>&1 || { echo "tune rc=$?"; tail -20 $OUT/tune_pipe.log; exit 1; }
tail -3 $OUT/tune_pipe.log
