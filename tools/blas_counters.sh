#!/bin/bash
# hipBLASLt vs dfu on the ViT shapes (via gpurun): per case the
# unprofiled times, hipBLASLt's kernel names (kernel trace), and the same two --pmc passes as
# tools/gemm_counters_r3.sh for both libraries.  tools/gemm_counters_summary.py reads the dirs.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/${CTR:-blasctr}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
PA="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"
PB="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_MFMA"
: > $OUT/times.txt
for c in ${CASES:-fc2_fwd fc1_fwd qkv_fwd fc1_dgrad_t qkv_dgrad_t}; do
  timeout -k 10 120 python3 $R/tools/blas_one.py $c --iters 30 >> $OUT/times.txt 2>&1 || { echo "blas time $c rc=$?"; exit 1; }
  timeout -k 10 120 python3 $R/tools/gemm_one.py $c --iters 30 >> $OUT/times.txt 2>&1 || { echo "dfu time $c rc=$?"; exit 1; }
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/${c}_blas_kt -o k -- python3 $R/tools/blas_one.py $c --iters 5 > /dev/null 2>&1 || { echo "kt $c rc=$?"; exit 1; }
  for lib in blas gemm; do
    timeout -s KILL 120 rocprofv3 --pmc $PA --output-format csv -d $OUT/${c}_${lib}_a -o c -- python3 $R/tools/${lib}_one.py $c --iters 5 > /dev/null 2>&1 || { echo "pass A $lib $c rc=$?"; exit 1; }
    timeout -s KILL 120 rocprofv3 --pmc $PB --output-format csv -d $OUT/${c}_${lib}_b -o c -- python3 $R/tools/${lib}_one.py $c --iters 5 > /dev/null 2>&1 || { echo "pass B $lib $c rc=$?"; exit 1; }
  done
  echo "$c done"
done
cat $OUT/times.txt
