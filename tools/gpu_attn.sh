#!/bin/bash
# attention backward variants: correctness + standalone timing per library (DFU_HIP_LIB)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
for lib in "" ${LIBS}; do
  export DFU_HIP_LIB=$lib
  timeout -k 10 200 python -u -m pytest "tests/test_kernels_gpu.py::test_attention" tests/test_fp16_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/attn_t.log 2>&1 || { echo "tests rc=$? ($lib)"; tail -30 $OUT/attn_t.log; exit 1; }
  echo "lib=${lib:-default}: $(tail -1 $OUT/attn_t.log)"
  for i in 1 2; do timeout -k 10 120 python tools/attn_time.py 2>/dev/null || exit 1; done
done
