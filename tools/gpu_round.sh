#!/bin/bash
# The round's measurement pass (via gpurun): smoke, the default bench line, the single-branch and
# Grad-CAM configs, kernel-trace profile + PMC traffic of the default (parity) step, per-shape
# GEMM table.  Summaries: tools/prof_summary.py, tools/pmc_by_kernel.py -> profiles/.
#   bash tools/gpu_round.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; OUT=$R/gpurun_out; TAG=${1:-r17}; mkdir -p $OUT; cd $R
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1 || { echo "smoke rc=$?"; tail -20 $OUT/smoke_$TAG.log; exit 1; }
tail -2 $OUT/smoke_$TAG.log
timeout -k 10 900 python bench.py > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { echo "bench rc=$?"; tail -20 $OUT/bench_$TAG.err; exit 1; }
cat $OUT/bench_$TAG.json
for c in rgb thermal; do
  timeout -k 10 400 python bench.py --config $c --no-cpu-baseline > $OUT/bench_${TAG}_$c.json 2> $OUT/bench_${TAG}_$c.err || { echo "bench $c rc=$?"; tail -20 $OUT/bench_${TAG}_$c.err; exit 1; }
done
timeout -k 10 600 python bench.py --config gradcam > $OUT/bench_${TAG}_gradcam.json 2> $OUT/bench_${TAG}_gradcam.err || { echo "bench gradcam rc=$?"; tail -20 $OUT/bench_${TAG}_gradcam.err; exit 1; }
timeout -k 10 300 python tools/gemm_step_profile.py > $OUT/gemm_step_$TAG.log 2>&1 || { echo "shapes rc=$?"; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o bench -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-alt-precision --no-parity > $OUT/prof_${TAG}_bench.json 2> $OUT/prof_${TAG}_bench.err || { echo "rocprof trace rc=$?"; tail -5 $OUT/prof_${TAG}_bench.err; exit 1; }
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmcf_$TAG -o pmc -- python3 $R/bench.py --steps 1 --warmup 1 --no-graph --no-cpu-baseline --no-alt-precision --no-parity > $OUT/pmcf_$TAG.log 2>&1 || { echo "pmc fetch rc=$?"; tail -5 $OUT/pmcf_$TAG.log; exit 1; }
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmcw_$TAG -o pmc -- python3 $R/bench.py --steps 1 --warmup 1 --no-graph --no-cpu-baseline --no-alt-precision --no-parity > $OUT/pmcw_$TAG.log 2>&1 || { echo "pmc write rc=$?"; tail -5 $OUT/pmcw_$TAG.log; exit 1; }
echo measure-done
