#!/bin/bash
# HIP runtime graph-executor knobs vs eager at bert-base B = 32 (seq/s, ms/step; bench.py --steps 30 --warmup 5).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
out=gpurun_out/graph_env_r5.log
: > $out
run() {  # $1 = label, rest = env assignments
  local lab=$1; shift
  v=$(env "$@" timeout -k 10 300 python bench.py --steps 30 --warmup 5 ${ARGS:---batch_size 32} $GFLAG 2>/dev/null | tail -1 | python -c "import json,sys; j=json.loads(sys.stdin.read()); print(j['value'], j['ms_per_step'])") || exit 1
  echo "$lab : $v" | tee -a $out
}
for r in 1 2; do
  GFLAG= run eager HSD_X=0
  GFLAG=--hip_graph run graph_default HSD_X=0
  GFLAG=--hip_graph run graph_pktcap0 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
  GFLAG=--hip_graph run graph_pktcap1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=1
  GFLAG=--hip_graph run graph_queues1 DEBUG_HIP_FORCE_GRAPH_QUEUES=1
  GFLAG=--hip_graph run graph_queues2 DEBUG_HIP_FORCE_GRAPH_QUEUES=2
  GFLAG=--hip_graph run graph_queues4 DEBUG_HIP_FORCE_GRAPH_QUEUES=4
  GFLAG=--hip_graph run graph_batch64 DEBUG_HIP_GRAPH_BATCH_SIZE=64
  GFLAG=--hip_graph run graph_batch1 DEBUG_HIP_GRAPH_BATCH_SIZE=1
done
