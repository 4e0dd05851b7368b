#!/bin/bash
# L2 / clock counter passes for single GEMMs (tools/gemm_one.py) on the GPU box: SQ busy/wait
# and MFMA cycles with GRBM_GUI_ACTIVE (clock), L2 hit/miss, and FETCH_SIZE, one pass each.
#   bash tools/gemm_l2_counters.sh fc1_fwd:13 fc2_fwd:13 ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/l2ctr
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
PA="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"
for spec in "$@"; do
  case_=${spec%:*}; tile=${spec#*:}
  timeout -k 10 120 python3 $R/tools/gemm_one.py $case_ --tile $tile --iters 20 >> $OUT/times.txt 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc $PA --output-format csv -d $OUT/${case_}_t${tile}_a -o c -- python3 $R/tools/gemm_one.py $case_ --tile $tile --iters 5 > /dev/null 2>&1 || { echo "pass A rc=$?"; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/${case_}_t${tile}_b -o c -- python3 $R/tools/gemm_one.py $case_ --tile $tile --iters 5 > /dev/null 2>&1 || { echo "pass B rc=$?"; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/${case_}_t${tile}_c -o c -- python3 $R/tools/gemm_one.py $case_ --tile $tile --iters 5 > /dev/null 2>&1 || { echo "pass C rc=$?"; exit 1; }
done
cat $OUT/times.txt
