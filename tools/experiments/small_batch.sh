#!/bin/bash
# Small-batch configs (the reference's own bert-large S=512 per-rank B=8, and bert-base S=128 B=32..256) under
# the 256x256 gemm2 body vs the 256x128 two-workgroups-per-CU gemm3 body (HSD_GEMM3 bit 0 = NT, bit 1 = TT).
# Usage (GPU box): bash tools/small_batch.sh > gpurun_out/small_batch.log
set -e
run() {
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 "$@" | grep '"metric"' | python -c \
    'import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({"model": d["config"]["model"], "B": d["config"]["global_batch"], "S": d["config"]["seq_len"], "seq_s": d["value"], "ms": d["ms_per_step"]}))'
}
for cfg in "--model bert-large-uncased --seq_len 512 --batch_size 8" "--model bert-large-uncased --seq_len 512 --batch_size 16" \
           "--batch_size 32" "--batch_size 64" "--batch_size 128" "--batch_size 256"; do
  for g3 in 0 1 3; do
    echo -n "gemm3=$g3 "
    HSD_GEMM3=$g3 run $cfg
  done
done
