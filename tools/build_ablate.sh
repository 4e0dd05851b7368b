#!/bin/bash
# Experiment builds of the persistent phased GEMM: for each mask, gemm_ps.hip compiled with
# -DDFU_PS_ABLATE=<mask> (timing ablations: results wrong by design), linked with the product
# objects into dfu_hip/libdfu_ablate_<mask>.so (select with DFU_HIP_LIB=...).
#   bash tools/build_ablate.sh 1 5 13 ...
set -e
cd "$(dirname "$0")/../dfu-multimodal_amd"
make -j8 >/dev/null
for m in "$@"; do
  SRC=gemm_ps
  DEF=-DDFU_PS_ABLATE=$m
  OBJS=$(ls build/*.o | grep -v $SRC.hip.o)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $DEF \
      -c csrc/$SRC.hip -o build/ablate_$m.o.tmp
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o dfu_hip/libdfu_ablate_$m.so \
      $OBJS build/ablate_$m.o.tmp
  rm -f build/ablate_$m.o.tmp
done
