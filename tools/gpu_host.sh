#!/bin/bash
# host enqueue time and bench A/B of host-side changes (env toggles in AB)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
for ab in ${AB}; do
  env ${ab//:/ } timeout -k 10 200 python tools/host_step_time.py --steps 20 > $OUT/host_$ab.txt 2>&1 || { echo "host rc=$?"; tail -5 $OUT/host_$ab.txt; exit 1; }
  echo "$ab"; tail -2 $OUT/host_$ab.txt
done
REPS=${REPS:-2} STEPS=30 EXTRA="--no-alt-precision --no-parity" bash tools/gpu_ab.sh
