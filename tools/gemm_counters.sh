#!/bin/bash
# SQ counter passes for single GEMMs (tools/gemm_one.py) on the GPU box.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/ctr
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
PA="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
PB="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_MFMA"
for spec in "$@"; do
  case_=${spec%:*}; tile=${spec#*:}
  timeout -k 10 120 python3 $R/tools/gemm_one.py $case_ --tile $tile --iters 20 >> $OUT/times.txt 2>&1 || exit 1
  timeout -k 10 180 rocprofv3 --pmc $PA --output-format csv -d $OUT/${case_}_t${tile}_a -o c -- python3 $R/tools/gemm_one.py $case_ --tile $tile --iters 5 > /dev/null 2>&1 || { echo "pass A rc=$?"; exit 1; }
  timeout -k 10 180 rocprofv3 --pmc $PB --output-format csv -d $OUT/${case_}_t${tile}_b -o c -- python3 $R/tools/gemm_one.py $case_ --tile $tile --iters 5 > /dev/null 2>&1 || { echo "pass B rc=$?"; exit 1; }
done
cat $OUT/times.txt
