#!/bin/bash
# Same-box A/B of bench lines under env toggles, alternating, REPS rounds.
#   AB="DFU_X=0 DFU_X=1 DFU_X=1:DFU_Y=2"  (variants by spaces; ":" joins variables of one variant)
#   CONFIG=fusion REPS=3 bash tools/gpu_ab.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
for rep in $(seq ${REPS:-3}); do
  for ab in ${AB}; do
    env ${ab//:/ } timeout -k 10 300 python bench.py --config ${CONFIG:-fusion} --no-cpu-baseline ${EXTRA:---no-alt-precision} --steps ${STEPS:-30} > $OUT/ab.json 2> $OUT/ab.err || { echo "bench rc=$?"; tail -20 $OUT/ab.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/ab.json')); print('$ab', 'rep$rep', d['value'], d.get('gpu_step_ms',{}).get('median'), d.get('roofline',{}).get('achieved'), (d.get('precision_modes') or {}).get('bf16x3',{}).get('ms_per_step'))"
  done
done
