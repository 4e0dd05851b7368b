#!/bin/bash
# Round-3 pass (via gpurun): the new / changed GPU tests, the C3 bench line (in-run parity,
# physical-core CPU baseline) and the C5 Grad-CAM line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
TAG=${1:-r3a}
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread ${TESTS:-tests/test_dropin_gpu.py tests/test_loop_gpu.py tests/test_streams_gpu.py} > $OUT/t_$TAG.log 2>&1 || { echo "pytest rc=$?"; tail -40 $OUT/t_$TAG.log; exit 1; }
grep -E "PASS|FAIL|\[" $OUT/t_$TAG.log | tail -30
timeout -k 10 400 python bench.py --steps 20 > $OUT/b_${TAG}.json 2> $OUT/b_${TAG}.err || { echo "bench rc=$?"; tail -20 $OUT/b_${TAG}.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/b_${TAG}.json')); print(d['value'], d['precision_modes'], d['parity'], d['cpu_baseline'])"
timeout -k 10 300 python bench.py --config gradcam --steps 20 --no-cpu-baseline > $OUT/b_${TAG}_gc.json 2> $OUT/b_${TAG}_gc.err || { echo "bench gc rc=$?"; tail -20 $OUT/b_${TAG}_gc.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/b_${TAG}_gc.json')); print(d['value'], d['ms_per_step'], d['config'])"
echo done
