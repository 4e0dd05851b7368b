#!/bin/bash
# Same-box A/B of the bench step under environment settings (one bench process per setting,
# alternating, N rounds).  bash tools/gpu_ab_env.sh <tag> <rounds> "<env A>" "<env B>" ...
#   e.g. bash tools/gpu_ab_env.sh beside 3 "DFU_RESNET_WGRAD_BESIDE=0" "DFU_RESNET_WGRAD_BESIDE=1"
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; OUT=$R/gpurun_out; TAG=$1; N=$2; shift 2; mkdir -p $OUT; cd $R
ARGS="--no-alt-precision --no-parity --no-cpu-baseline --steps 30 --warmup 5 $BENCH_EXTRA"
for i in $(seq 1 $N); do
  k=0
  for e in "$@"; do
    k=$((k + 1))
    env $e timeout -k 10 300 python bench.py $ARGS > $OUT/abe_${TAG}_${k}_$i.json 2> $OUT/abe_${TAG}_${k}_$i.err || { echo "[$e] rc=$?"; tail -5 $OUT/abe_${TAG}_${k}_$i.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/abe_${TAG}_${k}_$i.json')); print('[$e]', $i, d['value'], d['ms_per_step'], d['gpu_step_ms']['median'])"
  done
done
