#!/bin/bash
# Same-box A/B of the bench: each argument is "NAME:ENV=VAL,..." ; runs bench.py per variant.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
CFG=${CFG:-fusion}
for spec in "$@"; do
  name=${spec%%:*}; envs=${spec#*:}
  [ "$envs" = "$spec" ] && envs=""
  env $(echo $envs | tr ',' ' ') timeout -k 10 300 python bench.py --config $CFG --no-cpu-baseline --no-alt-precision --steps 30 --warmup 5 > gpurun_out/ab_$name.json 2> gpurun_out/ab_$name.err || { echo "$name rc=$?"; tail -5 gpurun_out/ab_$name.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_$name.json').read().strip().splitlines()[-1]); print('$name', d['value'], d.get('gpu_step_ms'))"
done
