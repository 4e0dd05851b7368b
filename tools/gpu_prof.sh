#!/bin/bash
# Kernel-trace profile of the default bench step (C3, library-default precision) for the
# trace tools (tools/trace_phases.py, trace_gaps.py, trace_fill.py, prof_summary.py).
#   bash tools/gpu_prof.sh <tag> [extra bench.py args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; OUT=$R/gpurun_out; TAG=${1:-r20}; shift; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o bench -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-alt-precision --no-parity "$@" > $OUT/prof_${TAG}_bench.json 2> $OUT/prof_${TAG}_bench.err || { echo "rocprof trace rc=$?"; tail -5 $OUT/prof_${TAG}_bench.err; exit 1; }
cat $OUT/prof_${TAG}_bench.json
find $OUT/prof_$TAG -name "*.csv" | head
