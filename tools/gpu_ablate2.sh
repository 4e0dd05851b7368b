#!/bin/bash
# Compile-time ablations of the persistent phased GEMM (tools/build_ablate.sh libraries).
#   MASKS="0 1 5 13" bash tools/gpu_ablate2.sh fc1_fwd:13 fc2_fwd:13
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
for spec in "$@"; do
  case_=${spec%:*}; tile=${spec#*:}
  for m in ${MASKS:-0}; do
    lib=$R/dfu-multimodal_amd/dfu_hip/libdfu_ablate_$m.so
    [ "$m" = 0 ] && lib=$R/dfu-multimodal_amd/dfu_hip/libdfu_hip.so
    echo -n "mask $m: " >> $OUT/ablate2.txt
    DFU_HIP_LIB=$lib timeout -k 10 60 python3 tools/gemm_one.py $case_ --tile $tile --iters 20 2>/dev/null >> $OUT/ablate2.txt || exit 1
  done
done
cat $OUT/ablate2.txt
