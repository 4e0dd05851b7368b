set -o pipefail
OUT=gpurun_out
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-alt-precision --no-parity --no-cpu-baseline --steps 30 --warmup 5 --graph > $OUT/g_$i.json 2>$OUT/g_$i.err || exit 1
  python -c "import json; d=json.load(open('$OUT/g_$i.json')); print('graph', d['value'], d['ms_per_step'], d['gpu_step_ms']['median'], d['config'].get('hip_graph'))"
  timeout -k 10 300 python bench.py --no-alt-precision --no-parity --no-cpu-baseline --steps 30 --warmup 5 > $OUT/e_$i.json 2>$OUT/e_$i.err || exit 1
  python -c "import json; d=json.load(open('$OUT/e_$i.json')); print('eager', d['value'], d['ms_per_step'], d['gpu_step_ms']['median'])"
done
timeout -k 10 300 python tools/host_step_time.py --steps 20 > $OUT/host_r24.txt 2>&1 || exit 1
tail -3 $OUT/host_r24.txt
timeout -k 10 300 python tools/host_step_time.py --profile > $OUT/host_prof_r24.txt 2>&1 || exit 1
head -50 $OUT/host_prof_r24.txt
