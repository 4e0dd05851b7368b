#!/bin/bash
# Same-box A/B of bench lines under env toggles (via gpurun):
#   AB="DFU_X=0 DFU_X=1" CONFIGS="fusion" REPS=2 bash tools/gpu_ab.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
TAG=${1:-ab}
mkdir -p $OUT
cd $R
for c in ${CONFIGS:-fusion}; do
  for rep in $(seq 1 ${REPS:-2}); do
    for ab in ${AB:-NONE=1}; do
      env $ab timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-alt-precision --no-parity --steps ${STEPS:-30} ${EXTRA:-} > $OUT/ab_${TAG}.json 2> $OUT/ab_${TAG}.err || { echo "bench rc=$?"; tail -20 $OUT/ab_${TAG}.err; exit 1; }
      python -c "import json; d=json.load(open('$OUT/ab_${TAG}.json')); print('$c', '$ab', 'rep$rep', d['value'], d['gpu_step_ms']['median'])"
    done
  done
done
echo ab-done
