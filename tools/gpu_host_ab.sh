#!/bin/bash
# Host-enqueue A/B of the eager fusion step: ab_old/ (a `git archive` of the baseline commit with
# the current libdfu_hip.so copied in) against this tree, alternating, then the GPU suite and the
# host profile of this tree.  Run through gpurun from the repo root.
set -e
mkdir -p gpurun_out
for r in 1 2 3; do
  (cd ab_old && timeout -k 10 240 python -u tools/host_step_time.py --steps 60 --pin) > gpurun_out/hst_old_$r.txt 2>&1
  timeout -k 10 240 python -u tools/host_step_time.py --steps 60 --pin > gpurun_out/hst_new_$r.txt 2>&1
done
grep -H "host total\|host fastest" gpurun_out/hst_old_*.txt gpurun_out/hst_new_*.txt
[ "${SUITE:-1}" = 0 ] && exit 0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_host.txt 2>&1
tail -2 gpurun_out/gpu_tests_host.txt
timeout -k 10 300 python -u tools/host_breakdown.py > gpurun_out/host_breakdown_new.txt 2>&1
