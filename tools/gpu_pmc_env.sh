#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (separate runs) of one bench step under an environment setting,
# summarised per kernel (tools/pmc_by_kernel.py).  bash tools/gpu_pmc_env.sh <tag> "<VAR=value ...>"
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; OUT=$R/gpurun_out; TAG=$1; mkdir -p $OUT
for kv in $2; do export "$kv"; done
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 1 --warmup 1 --no-graph --no-cpu-baseline --no-alt-precision --no-parity"
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmcf_$TAG -o pmc -- python3 $R/bench.py $ARGS > $OUT/pmcf_$TAG.log 2>&1 || { echo "pmc fetch rc=$?"; tail -5 $OUT/pmcf_$TAG.log; exit 1; }
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmcw_$TAG -o pmc -- python3 $R/bench.py $ARGS > $OUT/pmcw_$TAG.log 2>&1 || { echo "pmc write rc=$?"; tail -5 $OUT/pmcw_$TAG.log; exit 1; }
python3 $R/tools/pmc_by_kernel.py $OUT/pmcf_$TAG/pmc_counter_collection.csv $OUT/pmcw_$TAG/pmc_counter_collection.csv > $OUT/pmc_by_kernel_$TAG.txt
head -14 $OUT/pmc_by_kernel_$TAG.txt
