#!/bin/bash
# One build-measure iteration on the GPU box: the named GPU tests, smoke, then the default bench
# line (C3, library-default precision).  bash tools/gpu_iter.sh <tag> "<pytest -k expr or files>"
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; OUT=$R/gpurun_out; TAG=${1:-it}; mkdir -p $OUT; cd $R
if [ -n "$2" ]; then
  timeout -k 10 600 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread $2 > $OUT/t_$TAG.log 2>&1 || { echo "tests rc=$?"; tail -40 $OUT/t_$TAG.log; exit 1; }
  tail -3 $OUT/t_$TAG.log
fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1 || { echo "smoke rc=$?"; tail -20 $OUT/smoke_$TAG.log; exit 1; }
tail -3 $OUT/smoke_$TAG.log
timeout -k 10 600 python bench.py ${BENCH_ARGS:---no-cpu-baseline} > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { echo "bench rc=$?"; tail -20 $OUT/bench_$TAG.err; exit 1; }
python -c "
import json; d=json.load(open('$OUT/bench_$TAG.json'))
print('value', d['value'], 'ms', d['ms_per_step'], 'gpu median', d['gpu_step_ms']['median'], 'modes', {k: v['value'] for k, v in d['precision_modes'].items()}, 'parity', {k: v['max_abs_logits_vs_fp32_oracle'] for k, v in (d['parity'] or {}).items() if isinstance(v, dict)}, 'gemm', d['roofline']['achieved'], d['roofline']['avg_launch_us'])"
