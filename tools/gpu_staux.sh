set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out; rm -f gpurun_out/ablate2.txt
MASKS="0 a2 a1 a3 a18 0" bash tools/gpu_ablate2.sh qkv_fwd:8 fc1_gelu:8 fc2_fwd_resid:8 fc1_fwd:8 > /dev/null || exit 1
cat gpurun_out/ablate2.txt
for m in 0 a2 0 a2; do
  lib=$R/dfu-multimodal_amd/dfu_hip/libdfu_ablate_$m.so; [ "$m" = 0 ] && lib=$R/dfu-multimodal_amd/dfu_hip/libdfu_hip.so
  DFU_HIP_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-alt-precision --steps 30 > gpurun_out/b_$m.json 2> gpurun_out/b_$m.err || { tail gpurun_out/b_$m.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/b_$m.json')); print('$m', d['value'], d['gpu_step_ms'])"
done
