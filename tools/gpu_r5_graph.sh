#!/bin/bash
# Eager vs whole-step HIP graph at small batches: throughput A/B and per-kernel stats of both (kernel trace only).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/gr5
for r in 1 2; do
  for a in "--batch_size 32" "--batch_size 32 --hip_graph" "--model bert-large-uncased --seq_len 512 --batch_size 8" "--model bert-large-uncased --seq_len 512 --batch_size 8 --hip_graph"; do
    v=$(timeout -k 10 300 python bench.py --steps 30 --warmup 5 $a 2>/dev/null | tail -1 | python -c "import json,sys; j=json.loads(sys.stdin.read()); print(j['value'], j['ms_per_step'])") || exit 1
    echo "$a : $v" | tee -a gpurun_out/graph_r5.log
  done
done
for m in eager graph; do
  f=""; [ $m = graph ] && f="--hip_graph"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/gr5/$m -o run -- python bench.py --steps 13 --warmup 3 --batch_size 32 $f > gpurun_out/gr5_$m.log 2>&1 || exit 1
done
