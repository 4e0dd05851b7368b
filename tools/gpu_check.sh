set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 600 python -u -m pytest -s -q --timeout 300 --timeout-method thread tests/test_configs_gpu.py tests/test_dropin_gpu.py tests/test_gradcam_gpu.py tests/test_eval_gpu.py tests/test_parallel_gpu.py > $OUT/t2.log 2>&1 || { echo "tests rc=$?"; tail -30 $OUT/t2.log; exit 1; }
grep -E "^\[|^  |passed|failed" $OUT/t2.log | head -60
for c in thermal rgb; do
  timeout -k 10 400 python bench.py --config $c --no-cpu-baseline > $OUT/b2_$c.json 2> $OUT/b2_$c.err || { echo "bench $c rc=$?"; tail -20 $OUT/b2_$c.err; exit 1; }
  cat $OUT/b2_$c.json
done
timeout -k 10 600 python bench.py --config gradcam --no-cpu-baseline > $OUT/b2_gradcam.json 2> $OUT/b2_gradcam.err || { echo "bench gradcam rc=$?"; tail -20 $OUT/b2_gradcam.err; exit 1; }
cat $OUT/b2_gradcam.json
