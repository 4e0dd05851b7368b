#!/bin/bash
# parity-mode step profile (via gpurun): rocprofv3 kernel trace + stats of the default bench
# (parity mode only, no CPU legs)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
TAG=${1:-par}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o bench -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-alt-precision --no-parity > $OUT/prof_${TAG}_bench.json 2> $OUT/prof_${TAG}_bench.err || { echo "rocprof rc=$?"; tail -5 $OUT/prof_${TAG}_bench.err; exit 1; }
ls -R $OUT/prof_$TAG | head
echo done
