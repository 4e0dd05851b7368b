#!/bin/bash
# Experiment build of one translation unit with extra defines, linked with the product objects
# into dfu_hip/libdfu_exp_<tag>.so (select at run time with DFU_HIP_LIB=...).
#   bash tools/build_exp.sh <tag> <source stem> "-DMACRO=1 ..."
set -e
cd "$(dirname "$0")/../dfu-multimodal_amd"
make -j8 >/dev/null
TAG=$1; SRC=$2; DEF=$3
OBJS=$(ls build/*.o | grep -v "/$SRC.hip.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $DEF -c csrc/$SRC.hip -o build/exp_$TAG.o.tmp
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o dfu_hip/libdfu_exp_$TAG.so $OBJS build/exp_$TAG.o.tmp
rm -f build/exp_$TAG.o.tmp
