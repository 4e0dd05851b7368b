#!/bin/bash
# Per-shape GEMM table with PMC HBM bytes (tools/gemm_shape_traffic.py): the recorded step's
# distinct GEMMs replayed between markers under separate FETCH_SIZE / WRITE_SIZE passes, times
# from an unprofiled run.  bash tools/gpu_shape_traffic.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; OUT=$R/gpurun_out; TAG=${1:-r25}; mkdir -p $OUT; cd $R
timeout -k 10 300 python tools/gemm_step_profile.py --iters 5 > $OUT/shape_times_$TAG.txt 2>&1 || { echo "times rc=$?"; tail -5 $OUT/shape_times_$TAG.txt; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/spf_$TAG -o pmc -- python3 $R/tools/gemm_step_profile.py --iters 5 --markers $OUT/shapes_$TAG.json > $OUT/spf_$TAG.log 2>&1 || { echo "fetch rc=$?"; tail -5 $OUT/spf_$TAG.log; exit 1; }
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/spw_$TAG -o pmc -- python3 $R/tools/gemm_step_profile.py --iters 5 --markers $OUT/shapes_$TAG.json > $OUT/spw_$TAG.log 2>&1 || { echo "write rc=$?"; tail -5 $OUT/spw_$TAG.log; exit 1; }
python3 $R/tools/gemm_shape_traffic.py $OUT/shapes_$TAG.json $OUT/spf_$TAG/pmc_counter_collection.csv $OUT/spw_$TAG/pmc_counter_collection.csv $OUT/shape_times_$TAG.txt > $OUT/shape_traffic_$TAG.md
head -50 $OUT/shape_traffic_$TAG.md
