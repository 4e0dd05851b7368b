#!/bin/bash
# bf16x3 step profile (via gpurun): bench line of both modes, then a rocprofv3 kernel trace of
# the bf16x3 fusion step.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
TAG=${1:-x3}
mkdir -p $OUT
cd $R
timeout -k 10 300 python bench.py --precision bf16x3 --no-cpu-baseline --steps 20 > $OUT/b_${TAG}.json 2> $OUT/b_${TAG}.err || { echo "bench rc=$?"; tail -20 $OUT/b_${TAG}.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/b_${TAG}.json')); print(d['precision_modes'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o bench -- python3 $R/bench.py --precision bf16x3 --steps 10 --warmup 3 --no-cpu-baseline --no-alt-precision > $OUT/prof_${TAG}_bench.json 2> $OUT/prof_${TAG}_bench.err || { echo "rocprof rc=$?"; tail -5 $OUT/prof_${TAG}_bench.err; exit 1; }
echo done
