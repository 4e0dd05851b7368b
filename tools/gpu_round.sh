#!/bin/bash
# One GPU-box pass: GPU tests, smoke, rocprofv3 kernel stats of the bench (used via gpurun).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 900 python -m pytest tests -m gpu -q -s --maxfail=5 > $OUT/pytest_gpu.log 2>&1 || echo "pytest rc=$? (continuing)"
tail -3 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log | tail -2
