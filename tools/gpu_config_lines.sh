#!/bin/bash
# The default-precision parity tests with their printed numbers (C2, RGB-only, drop-in, Grad-CAM,
# eval, DP world 2), then the thermal / RGB / Grad-CAM bench lines.  bash tools/gpu_config_lines.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 600 python -u -m pytest -s -q --timeout 300 --timeout-method thread tests/test_configs_gpu.py tests/test_dropin_gpu.py tests/test_gradcam_gpu.py tests/test_eval_gpu.py tests/test_parallel_gpu.py > $OUT/t_cfg.log 2>&1 || { echo "tests rc=$?"; tail -30 $OUT/t_cfg.log; exit 1; }
grep -E "^\[|^  |passed|failed" $OUT/t_cfg.log | head -60
for c in thermal rgb; do
  timeout -k 10 400 python bench.py --config $c --no-cpu-baseline > $OUT/cfg_$c.json 2> $OUT/cfg_$c.err || { echo "bench $c rc=$?"; tail -20 $OUT/cfg_$c.err; exit 1; }
  cat $OUT/cfg_$c.json
done
timeout -k 10 600 python bench.py --config gradcam --no-cpu-baseline > $OUT/cfg_gradcam.json 2> $OUT/cfg_gradcam.err || { echo "bench gradcam rc=$?"; tail -20 $OUT/cfg_gradcam.err; exit 1; }
cat $OUT/cfg_gradcam.json
