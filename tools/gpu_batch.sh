#!/bin/bash
# One GPU-box pass after a batch of kernel changes: GPU tests, GEMM tile sweep, bench line,
# SQ counters on representative GEMMs.  Each GPU step has its own time limit; stops at the first
# failure of a correctness step.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 600 python -m pytest tests -m gpu -q -x -s > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || { echo "gpu tests rc=$rc"; grep -E "^E |FAILED|Error" $OUT/pytest_gpu.log | head -20; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { echo "bench rc=$?"; tail -5 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 python tools/gemm_bench.py --sweep > $OUT/gb.log 2>&1 || { echo "sweep rc=$?"; exit 1; }
bash tools/gemm_counters.sh fc1_fwd:5 fc1_fwd:4 l1c3_fwd:5 || exit 1
echo batch-done
