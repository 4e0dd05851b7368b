#!/bin/bash
# Per-config measurement pass (via gpurun): the C3 kernel-trace profile without the bf16x3
# timing, bench lines of the single-branch configs, and the per-shape GEMM table of the step.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
TAG=${1:-r05}
mkdir -p $OUT
cd $R
for c in rgb thermal; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-parity > $OUT/bench_${TAG}_$c.json 2> $OUT/bench_${TAG}_$c.err || { echo "bench $c rc=$?"; tail -20 $OUT/bench_${TAG}_$c.err; exit 1; }
  cat $OUT/bench_${TAG}_$c.json
done
timeout -k 10 300 python tools/gemm_step_profile.py > $OUT/gemm_step_$TAG.log 2>&1 || { echo "profile rc=$?"; tail -20 $OUT/gemm_step_$TAG.log; exit 1; }
timeout -k 10 300 python tools/gemm_step_profile.py --config rgb > $OUT/gemm_step_${TAG}_rgb.log 2>&1 || { echo "profile rgb rc=$?"; tail -20 $OUT/gemm_step_${TAG}_rgb.log; exit 1; }
cd /tmp && export TMPDIR=/tmp

timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_${TAG}_rgb -o bench -- python3 $R/bench.py --config rgb --steps 10 --warmup 3 --no-cpu-baseline --no-alt-precision --no-parity > $OUT/prof_${TAG}_rgb_bench.json 2> $OUT/prof_${TAG}_rgb_bench.err || { echo "rocprof rgb rc=$?"; tail -5 $OUT/prof_${TAG}_rgb_bench.err; exit 1; }
cd $R
timeout -k 10 300 python bench.py --config gradcam > $OUT/bench_${TAG}_gradcam.json 2> $OUT/bench_${TAG}_gradcam.err || { echo "bench gradcam rc=$?"; tail -20 $OUT/bench_${TAG}_gradcam.err; exit 1; }
cat $OUT/bench_${TAG}_gradcam.json
echo configs-done
