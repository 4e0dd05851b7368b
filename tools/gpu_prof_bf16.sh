#!/bin/bash
# rocprofv3 kernel trace of the default (bf16) bench step (via gpurun), for per-stream timelines.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
TAG=${1:-pb}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o bench -- python3 $R/bench.py --config ${CONFIG:-fusion} --steps 10 --warmup 3 --no-cpu-baseline --no-alt-precision --no-parity > $OUT/prof_${TAG}_bench.json 2> $OUT/prof_${TAG}_bench.err || { echo "rocprof rc=$?"; tail -5 $OUT/prof_${TAG}_bench.err; exit 1; }
echo done
