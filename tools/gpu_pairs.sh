#!/bin/bash
# Interleaved-pair bf16x3 GEMMs (dfu_gemm_desc.x3_pairs): precision tests, same-box A/B against
# the tripled K, per-shape GEMM tables both ways, and tuning of the pair GEMMs' plans.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_precision_gpu.py > $OUT/pairs_t.log 2>&1 || { echo "tests rc=$?"; tail -30 $OUT/pairs_t.log; exit 1; }
tail -2 $OUT/pairs_t.log
AB="DFU_X3_PAIRS=0 DFU_X3_PAIRS=1" REPS=${REPS:-3} bash tools/gpu_ab.sh || exit 1
for v in 0 1; do
  DFU_X3_PAIRS=$v timeout -k 10 300 python tools/gemm_step_profile.py --precision parity > $OUT/pairs_shapes_$v.log 2>&1 || { echo "shapes rc=$?"; tail -5 $OUT/pairs_shapes_$v.log; exit 1; }
done
cp dfu-multimodal_amd/csrc/gemm_tuned.inc $OUT/gemm_tuned.inc
timeout -k 10 600 python tools/gemm_tune.py --precision parity --only-x3-pairs --append --out $OUT/gemm_tuned.inc > $OUT/pairs_tune.log 2>&1 || { echo "tune rc=$?"; tail -5 $OUT/pairs_tune.log; exit 1; }
tail -3 $OUT/pairs_tune.log
echo pairs-done
