#!/bin/bash
# SQ counter passes over tools/attn_time.py (attention fwd + fused bwd) on the GPU box.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/actr
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
PA="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
PB="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_MFMA"
timeout -s KILL 120 rocprofv3 --pmc $PA --output-format csv -d $OUT/a -o c -- python3 $R/tools/attn_time.py > /dev/null 2>&1 || { echo "pass A rc=$?"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc $PB --output-format csv -d $OUT/b -o c -- python3 $R/tools/attn_time.py > /dev/null 2>&1 || { echo "pass B rc=$?"; exit 1; }
echo done
