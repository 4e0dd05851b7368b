#!/bin/bash
# GEMM tests, proj-forward tile check, kernel-trace profile of the bf16 fusion bench and the per-shape GEMM table.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gemm_persistent_gpu.py tests/test_kernels_gpu.py > gpurun_out/t_d.log 2>&1 || { tail -20 gpurun_out/t_d.log; exit 1; }
tail -1 gpurun_out/t_d.log
for t in 7 8; do timeout -k 10 60 python3 tools/gemm_one.py proj_fwd_resid --tile $t --check 2>/dev/null && timeout -k 10 60 python3 tools/gemm_one.py proj_fwd_resid --tile $t --iters 30 2>/dev/null || exit 1; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_${1:-p2} -o bench -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-alt-precision --no-parity > $R/gpurun_out/prof_${1:-p2}_bench.json 2> $R/gpurun_out/prof_${1:-p2}.err || exit 1
cd $R && timeout -k 10 300 python tools/gemm_step_profile.py > gpurun_out/shapes_${1:-p2}.txt 2>&1
