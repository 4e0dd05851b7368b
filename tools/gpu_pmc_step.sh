#!/bin/bash
# HBM bytes per kernel over one parity-mode fusion step: separate --pmc FETCH_SIZE / WRITE_SIZE
# passes of the same bench command (tools/pmc_by_kernel.py joins them on the CPU).
#   bash tools/gpu_pmc_step.sh <tag> [bench args...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; OUT=$R/gpurun_out; TAG=${1:-pmc}; shift; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d $OUT/${TAG}_$c -o pmc -- python3 $R/bench.py --steps 1 --warmup 1 --no-graph --no-cpu-baseline --no-alt-precision --no-parity "$@" > $OUT/${TAG}_$c.log 2>&1 || { echo "pmc $c rc=$?"; tail -5 $OUT/${TAG}_$c.log; exit 1; }
done
cd $R && python tools/pmc_by_kernel.py $OUT/${TAG}_FETCH_SIZE/pmc_counter_collection.csv $OUT/${TAG}_WRITE_SIZE/pmc_counter_collection.csv | head -45
