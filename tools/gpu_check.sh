#!/bin/bash
# Iteration pass (via gpurun): selected GPU tests, then bench lines (bf16 fusion with the x3 mode
# beside it, thermal-only, RGB-only) without the CPU baseline.
#   TESTS="tests/test_kernels_gpu.py" CONFIGS="fusion thermal" bash tools/gpu_check.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; OUT=$R/gpurun_out; TAG=${1:-c}; mkdir -p $OUT; cd $R
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu $TESTS > $OUT/t_$TAG.log 2>&1 || { echo "pytest rc=$?"; tail -30 $OUT/t_$TAG.log; exit 1; }
  tail -2 $OUT/t_$TAG.log
fi
for c in ${CONFIGS:-fusion}; do
  extra=""; [ "$c" != fusion ] && extra="--no-alt-precision"
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline $extra --steps ${STEPS:-30} > $OUT/b_${TAG}_$c.json 2> $OUT/b_${TAG}_$c.err || { echo "bench rc=$?"; tail -20 $OUT/b_${TAG}_$c.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/b_${TAG}_$c.json')); print('$c', d['value'], d.get('gpu_step_ms',{}).get('median'), d.get('roofline',{}).get('achieved'), d.get('precision_modes',{}).get('bf16x3'))"
done
