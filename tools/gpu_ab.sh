#!/bin/bash
# Same-box A/B of the bench step: ab_old/ (a copy of an earlier tree with its own built library,
# git-ignored) against this tree, alternating, N rounds.  bash tools/gpu_ab.sh <tag> [rounds]
# [extra bench args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; OUT=$R/gpurun_out; TAG=${1:-ab}; N=${2:-3}; shift 2; mkdir -p $OUT
ARGS="--no-alt-precision --no-parity --no-cpu-baseline --steps 30 --warmup 5 $*"
for i in $(seq 1 $N); do
  for side in old new; do
    if [ $side = old ]; then D=$R/ab_old; else D=$R; fi
    (cd $D && timeout -k 10 300 python bench.py $ARGS > $OUT/ab_${TAG}_${side}_$i.json 2> $OUT/ab_${TAG}_${side}_$i.err) || { echo "$side rc=$?"; tail -5 $OUT/ab_${TAG}_${side}_$i.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/ab_${TAG}_${side}_$i.json')); print('$side', $i, d['value'], d['ms_per_step'], d['gpu_step_ms']['median'])"
  done
done
