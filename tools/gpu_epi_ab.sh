set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; L=$R/dfu-multimodal_amd/dfu_hip
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gemm_persistent_gpu.py tests/test_kernels_gpu.py > gpurun_out/t_c.log 2>&1; tail -1 gpurun_out/t_c.log
for c in fc2_fwd_resid proj_fwd_resid fc2x3_fwd_resid; do for t in 8 9; do timeout -k 10 60 python3 tools/gemm_one.py $c --tile $t --check 2>/dev/null || { echo "check $c $t failed"; exit 1; }; done; done
for rep in 1 2; do for lib in libdfu_ablate_old.so libdfu_hip.so; do for c in fc2_fwd_resid:8 fc2x3_fwd_resid:9 fc2_dgrad_t:8 qkv_fwd:8 fc1_gelu:8; do
  DFU_HIP_LIB=$L/$lib timeout -k 10 60 python3 tools/gemm_one.py ${c%:*} --tile ${c#*:} --iters 30 2>/dev/null | sed "s/^/$lib /" || exit 1
done; done; done
AB="DFU_HIP_LIB=$L/libdfu_ablate_old.so DFU_HIP_LIB=$L/libdfu_hip.so" REPS=3 EXTRA=" " bash tools/gpu_ab.sh
