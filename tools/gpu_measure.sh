#!/bin/bash
# Measurement pass on the GPU box (via gpurun): bench line, kernel-trace stats, PMC traffic.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
TAG=${1:-r01}
mkdir -p $OUT
cd $R
timeout -k 10 600 python bench.py > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { echo "bench rc=$?"; tail -20 $OUT/bench_$TAG.err; exit 1; }
cat $OUT/bench_$TAG.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o bench -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-alt-precision --no-parity > $OUT/prof_${TAG}_bench.json 2> $OUT/prof_${TAG}_bench.err || { echo "rocprof trace rc=$?"; tail -5 $OUT/prof_${TAG}_bench.err; exit 1; }
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmcf_$TAG -o pmc -- python3 $R/bench.py --steps 1 --warmup 1 --no-graph --no-cpu-baseline --no-alt-precision --no-parity > $OUT/pmcf_$TAG.log 2>&1 || { echo "pmc fetch rc=$?"; tail -5 $OUT/pmcf_$TAG.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmcw_$TAG -o pmc -- python3 $R/bench.py --steps 1 --warmup 1 --no-graph --no-cpu-baseline --no-alt-precision --no-parity > $OUT/pmcw_$TAG.log 2>&1 || { echo "pmc write rc=$?"; tail -5 $OUT/pmcw_$TAG.log; exit 1; }
echo measure-done
