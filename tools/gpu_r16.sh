#!/bin/bash
# round 4: fp16 ViT forward ("parity" mode) -- kernel tests, model parity, the stage study, bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest tests/test_fp16_gpu.py -m gpu -v -s -x --timeout 200 --timeout-method thread > $OUT/r16_fp16_tests.log 2>&1 || { echo "fp16 tests rc=$?"; tail -40 $OUT/r16_fp16_tests.log; exit 1; }
tail -3 $OUT/r16_fp16_tests.log
timeout -k 10 500 python -u -m pytest tests/test_model_parity_gpu.py -m gpu -v -s -x --timeout 400 --timeout-method thread -k "parity or bf16x3" > $OUT/r16_parity_tests.log 2>&1 || { echo "parity tests rc=$?"; tail -40 $OUT/r16_parity_tests.log; }
grep -E "parity\]|bf16x3\]|passed|failed" $OUT/r16_parity_tests.log | tail -8
timeout -k 10 600 python -u tools/precision_policy_study.py --out $OUT/r16b_precision_study.json > $OUT/r16b_study.txt 2>&1 || { echo "study rc=$?"; tail -20 $OUT/r16b_study.txt; exit 1; }
tail -22 $OUT/r16b_study.txt
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/r16b_bench.json 2> $OUT/r16b_bench.err || { echo "bench rc=$?"; tail -20 $OUT/r16b_bench.err; exit 1; }
python -c "import json;d=json.loads(open('$OUT/r16b_bench.json').read().strip().splitlines()[-1]);print(d['value'],d['precision_modes'],d['parity'])"
