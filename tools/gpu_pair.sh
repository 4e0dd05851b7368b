#!/bin/bash
# round 4: split-pair ResNet bf16x3 activations -- kernel tests, model parity, bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest tests/test_precision_gpu.py "tests/test_kernels_gpu.py::test_attention" -m gpu -v -s -x --timeout 200 --timeout-method thread > $OUT/pair_tests.log 2>&1 || { echo "precision tests rc=$?"; tail -40 $OUT/pair_tests.log; exit 1; }
tail -3 $OUT/pair_tests.log
timeout -k 10 500 python -u -m pytest tests/test_model_parity_gpu.py -m gpu -v -s -x --timeout 400 --timeout-method thread > $OUT/pair_parity.log 2>&1 || { echo "parity tests rc=$?"; tail -40 $OUT/pair_parity.log; exit 1; }
grep -E "parity|bf16x3|passed|failed" $OUT/pair_parity.log | tail -12
timeout -k 10 120 python -u tools/attn_time.py || exit 1
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/pair_bench.json 2> $OUT/pair_bench.err || { echo "bench rc=$?"; tail -20 $OUT/pair_bench.err; exit 1; }
python -c "import json;d=json.loads(open('$OUT/pair_bench.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['precision_modes'],d['parity'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_pair -o bench -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-alt-precision --no-parity > $OUT/prof_pair_bench.json 2> $OUT/prof_pair_bench.err || { echo "rocprof rc=$?"; tail -5 $OUT/prof_pair_bench.err; exit 1; }
cd $R && python tools/trace_phases.py $OUT/prof_pair/bench_kernel_trace.csv | tail -5
