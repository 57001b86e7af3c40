#!/bin/bash
# HSD_COMPUTE_PRIO A/B: eager steps on a high-priority stream (critical path before side-stream workgroups)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/r4_prio_ab.log
for rep in 1 2; do
for cfg in "--model bert-large-uncased --seq_len 512 --batch_size 8" "--batch_size 32" "--batch_size 256"; do
  for pr in 0 1; do
    HSD_COMPUTE_PRIO=$pr timeout -k 10 200 python bench.py --steps 30 --warmup 5 $cfg > gpurun_out/prio_bench.log 2>&1 || { tail -20 gpurun_out/prio_bench.log; exit 1; }
    echo "$cfg PRIO=$pr : $(tail -1 gpurun_out/prio_bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a gpurun_out/r4_prio_ab.log
  done
done
done
