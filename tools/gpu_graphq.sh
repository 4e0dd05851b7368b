#!/bin/bash
# Graph replay of the C3 step under HIP's graph-execution queue settings against eager (same box).
#   bash tools/gpu_graphq.sh <rounds>
set -o pipefail
OUT=gpurun_out; N=${1:-1}; mkdir -p $OUT
ARGS="--no-alt-precision --no-parity --no-cpu-baseline --steps 30 --warmup 5"
run() {  # tag env... -- bench args
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py $ARGS $EXTRA > $OUT/gq_$tag.json 2> $OUT/gq_$tag.err || { echo "[$tag] rc=$?"; tail -5 $OUT/gq_$tag.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/gq_$tag.json')); print('[$tag]', d['value'], d['ms_per_step'], d['gpu_step_ms']['median'], d['config'].get('hip_graph'))"
}
for i in $(seq 1 $N); do
  EXTRA="" run eager_$i X=0
  EXTRA="--graph" run graph_$i X=0
  EXTRA="--graph" run graph_q2_$i DEBUG_HIP_FORCE_GRAPH_QUEUES=2
  EXTRA="--graph" run graph_q4_$i DEBUG_HIP_FORCE_GRAPH_QUEUES=4
  EXTRA="--graph" run graph_q2p0_$i DEBUG_HIP_FORCE_GRAPH_QUEUES=2 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
done
