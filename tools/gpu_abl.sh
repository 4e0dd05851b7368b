#!/bin/bash
# MASKS="0 32 1" bash tools/gpu_abl.sh shape:tile ...   (compile-time ablations, tools/build_ablate.sh)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out; rm -f gpurun_out/ablate2.txt
bash tools/gpu_ablate2.sh "$@" > /dev/null || exit 1
cat gpurun_out/ablate2.txt
