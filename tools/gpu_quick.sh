#!/bin/bash
# Quick iteration pass (via gpurun): selected GPU tests, then same-box A/B bench lines of the
# given configs under env toggles, then one rocprofv3 kernel-trace of the first config.
#   TESTS="tests/test_kernels_gpu.py -k bn" CONFIGS="rgb fusion" AB="DFU_X=0 DFU_X=1" tools/gpu_quick.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
TAG=${1:-q}
mkdir -p $OUT
cd $R
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread $TESTS > $OUT/t_$TAG.log 2>&1 || { echo "pytest rc=$?"; tail -30 $OUT/t_$TAG.log; exit 1; }
  tail -2 $OUT/t_$TAG.log
fi
for c in ${CONFIGS:-rgb}; do
  for ab in ${AB:-NONE=1}; do
    for rep in 1 2; do
      env $ab timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-alt-precision --steps ${STEPS:-30} > $OUT/b_${TAG}_${c}.json 2> $OUT/b_${TAG}_${c}.err || { echo "bench rc=$?"; tail -20 $OUT/b_${TAG}_${c}.err; exit 1; }
      python -c "import json,sys; d=json.load(open('$OUT/b_${TAG}_${c}.json')); print('$c', '$ab', 'rep$rep', d['value'], d['gpu_step_ms']['median'])"
    done
  done
done
if [ -n "$PROF" ]; then
  c=${CONFIGS%% *}; c=${c:-rgb}
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o bench -- python3 $R/bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline --no-alt-precision > $OUT/prof_${TAG}_bench.json 2> $OUT/prof_${TAG}_bench.err || { echo "rocprof rc=$?"; tail -5 $OUT/prof_${TAG}_bench.err; exit 1; }
fi
echo quick-done
