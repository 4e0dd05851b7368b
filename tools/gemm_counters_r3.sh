#!/bin/bash
# MFMA-utilisation evidence for the step's top GEMM shapes (via gpurun):
# per case the tuned plan's time (tools/gemm_one.py, tile 0 = the library's plan), then two
# rocprofv3 --pmc passes of its own: (A) wave cycles / waits / MFMA busy / clock, (B) LDS and
# instruction counts.  tools/gemm_counters_summary.py turns gpurun_out/ctr3 into a table.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/${CTR:-ctr3}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
PA="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"
PB="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_MFMA"
: > $OUT/times.txt
for c in ${CASES:-fc2_dgrad_t fc1_gelu fc2_fwd_resid fc2_wgrad fc1_wgrad fc1_dgrad_t qkv_wgrad qkv_dgrad_t qkv_fwd}; do
  timeout -k 10 120 python3 $R/tools/gemm_one.py $c --iters 20 >> $OUT/times.txt 2>&1 || { echo "time $c rc=$?"; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc $PA --output-format csv -d $OUT/${c}_a -o c -- python3 $R/tools/gemm_one.py $c --iters 5 > /dev/null 2>&1 || { echo "pass A $c rc=$?"; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc $PB --output-format csv -d $OUT/${c}_b -o c -- python3 $R/tools/gemm_one.py $c --iters 5 > /dev/null 2>&1 || { echo "pass B $c rc=$?"; exit 1; }
  echo "$c done"
done
cat $OUT/times.txt
