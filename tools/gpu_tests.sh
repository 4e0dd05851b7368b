#!/bin/bash
# GPU test pass on the GPU box (via gpurun): the -m gpu suite (verbose, prints kept), then smoke.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
SEL=${1:-tests}
timeout -k 10 1000 python -u -m pytest $SEL -m gpu -v -s -x --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
