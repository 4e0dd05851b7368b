#!/bin/bash
# Experiment build of the whole library with extra compile definitions, for same-box A/B runs:
#   bash tools/build_variant.sh prio -DDFU_GEMM_PRIO=1   ->  dfu_hip/libdfu_prio.so
# (run with DFU_HIP_LIB=$PWD/dfu-multimodal_amd/dfu_hip/libdfu_prio.so)
set -e
name=$1; shift
cd "$(dirname "$0")/../dfu-multimodal_amd"
make -j8 OBJDIR=build_$name LIB=dfu_hip/libdfu_$name.so EXTRA="$*" >/dev/null
echo dfu_hip/libdfu_$name.so
