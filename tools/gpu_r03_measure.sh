#!/bin/bash
# Measurement pass on the GPU box (via gpurun): bench line, kernel-trace stats, PMC traffic of
# the bench's GEMMs, and the per-shape GEMM table (times + PMC bytes per launch).
#   bash tools/gpu_r03_measure.sh <tag> [bench args...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
TAG=${1:-r03}
shift
mkdir -p $OUT
cd $R
timeout -k 10 400 python bench.py "$@" > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { echo "bench rc=$?"; tail -20 $OUT/bench_$TAG.err; exit 1; }
cat $OUT/bench_$TAG.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o bench -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-alt-precision "$@" > $OUT/prof_${TAG}_bench.json 2> $OUT/prof_${TAG}_bench.err || { echo "rocprof trace rc=$?"; tail -5 $OUT/prof_${TAG}_bench.err; exit 1; }
echo trace-done
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmcf_$TAG -o pmc -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-alt-precision "$@" > $OUT/pmcf_$TAG.log 2>&1 || { echo "pmc fetch rc=$?"; tail -5 $OUT/pmcf_$TAG.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmcw_$TAG -o pmc -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-alt-precision "$@" > $OUT/pmcw_$TAG.log 2>&1 || { echo "pmc write rc=$?"; tail -5 $OUT/pmcw_$TAG.log; exit 1; }
echo pmc-done
if [ -z "$NO_SHAPES" ]; then
timeout -k 10 300 python3 $R/tools/gemm_step_profile.py --iters 10 > $OUT/gemm_shapes_$TAG.txt 2>&1 || { echo "shape profile rc=$?"; tail -5 $OUT/gemm_shapes_$TAG.txt; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/spf_$TAG -o pmc -- python3 $R/tools/gemm_step_profile.py --iters 3 --markers $OUT/shapes_$TAG.json > $OUT/spf_$TAG.log 2>&1 || { echo "shape pmc fetch rc=$?"; tail -5 $OUT/spf_$TAG.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/spw_$TAG -o pmc -- python3 $R/tools/gemm_step_profile.py --iters 3 --markers $OUT/shapes_$TAG.json > $OUT/spw_$TAG.log 2>&1 || { echo "shape pmc write rc=$?"; tail -5 $OUT/spw_$TAG.log; exit 1; }
fi
echo measure-done
