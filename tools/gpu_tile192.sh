#!/bin/bash
# 192x256 persistent tile (tile 9) vs the 256x256 one (tile 8) on the N = 768 ViT GEMMs.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out
for c in qkv_dgrad_t fc1_dgrad_t proj_dgrad_t fc2_fwd_resid proj_fwd_resid fc2x3_fwd_resid projx3_fwd_resid fc1_dgrad; do
  for t in 8 9; do
    timeout -k 10 60 python3 tools/gemm_one.py $c --tile $t --check 2>/dev/null || { echo "check $c $t failed"; exit 1; }
  done
done
for rep in 1 2; do
for c in qkv_dgrad_t fc1_dgrad_t proj_dgrad_t fc2_fwd_resid proj_fwd_resid fc2x3_fwd_resid projx3_fwd_resid fc1_dgrad; do
  for t in 8 9 ${EXTRA}; do
    timeout -k 10 60 python3 tools/gemm_one.py $c --tile $t --iters 30 2>/dev/null || exit 1
  done
done
done
