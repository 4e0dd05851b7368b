#!/bin/bash
# A/B builds of the BatchNorm finalize kernels' block size: bn.hip with -DDFU_FIN_WAVES=<n>
# linked with the product objects into dfu_hip/libdfu_fin<n>.so (select with DFU_HIP_LIB=...).
#   bash tools/build_fin.sh 4 8
set -e
cd "$(dirname "$0")/../dfu-multimodal_amd"
make -j8 >/dev/null
for n in "$@"; do
  OBJS=$(ls build/*.o | grep -v bn.hip.o)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -DDFU_FIN_WAVES=$n \
      -c csrc/bn.hip -o build/fin_$n.o.tmp
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o dfu_hip/libdfu_fin$n.so \
      $OBJS build/fin_$n.o.tmp
  rm -f build/fin_$n.o.tmp
done
