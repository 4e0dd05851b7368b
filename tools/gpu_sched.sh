#!/bin/bash
# Schedule variants of the persistent GEMM (tools/build_ablate.sh s<mask> libraries): a
# correctness check of each, then timings.   VARS="s16 s32" SHAPES="qkv_fwd:8 ..." bash tools/gpu_sched.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out; rm -f gpurun_out/ablate2.txt
for v in ${VARS}; do
  for c in ${CHECKS:-qkv_fwd fc1_dgrad fc2_wgrad}; do
    DFU_HIP_LIB=$R/dfu-multimodal_amd/dfu_hip/libdfu_ablate_$v.so timeout -k 10 60 python3 tools/gemm_one.py $c --tile 8 --check 2>/dev/null || { echo "check $v $c failed"; exit 1; }
  done
done
MASKS="0 ${VARS} 0 ${VARS}" bash tools/gpu_ablate2.sh ${SHAPES} > /dev/null || exit 1
sort -s -k3,3 gpurun_out/ablate2.txt
