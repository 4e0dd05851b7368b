#!/bin/bash
# End-of-iteration pass (via gpurun): the full -m gpu suite + smoke, then the measurement pass
# (bench line, kernel-trace stats, PMC traffic) and the per-config bench lines and GEMM tables.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-r06}
cd $R
bash tools/gpu_tests.sh && bash tools/gpu_measure.sh $TAG && bash tools/gpu_configs.sh $TAG
