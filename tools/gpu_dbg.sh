#!/bin/bash
# GEMM timing ablations (DFU_GEMM_DEBUG: 1 no epilogue, 2 no MFMA, 4 no DMA) on single GEMMs.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
for c in qkv_fwd:5 qkv_fwd:1 qkv_fwd:4 fc2_fwd:5 proj_fwd:5 fc1_wgrad:5 l1c3_fwd:5; do
  case_=${c%:*}; tile=${c#*:}
  for d in 0 1 2 4 3 5 6 7; do
    echo -n "dbg=$d "; DFU_GEMM_DEBUG=$d timeout -k 10 60 python tools/gemm_one.py $case_ --tile $tile --iters 30 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
