#!/bin/bash
# rocprofv3 kernel stats of bench.py for several env variants (same box): NAME:ENV=VAL,...
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
CFG=${CFG:-rgb}
cd /tmp && export TMPDIR=/tmp
for spec in "$@"; do
  name=${spec%%:*}; envs=${spec#*:}
  [ "$envs" = "$spec" ] && envs=""
  for kv in $(echo $envs | tr ',' ' '); do export "$kv"; done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pab_$name -o k -- python3 $R/bench.py --config $CFG --steps 10 --warmup 3 --no-cpu-baseline --no-alt-precision > $R/gpurun_out/pab_$name.log 2>&1 || { echo "$name rc=$?"; tail -5 $R/gpurun_out/pab_$name.log; exit 1; }
done
