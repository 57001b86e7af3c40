#!/bin/bash
# Small-batch configs with and without HIP-graph replay of forward + backward (bench.py --hip_graph, N = 1).
# Usage (GPU box): bash tools/small_batch_graph.sh > gpurun_out/small_batch_graph.log
set -e
run() {
  timeout -k 10 180 python bench.py --steps 20 --warmup 5 "$@" | grep '"metric"' | python -c \
    'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(json.dumps({"model": c["model"], "B": c["global_batch"], "S": c["seq_len"], "graph": c.get("hip_graph"), "seq_s": d["value"], "ms": d["ms_per_step"]}))'
}
for cfg in "--model bert-large-uncased --seq_len 512 --batch_size 8" "--batch_size 32" "--batch_size 64" "--batch_size 256"; do
  for g in "" "--hip_graph"; do
    HSD_GEMM3=${G3:-0} run $cfg $g
  done
done
