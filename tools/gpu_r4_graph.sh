#!/bin/bash
# Captured step with the wgrad side stream as a graph branch: graph tests, then graph vs eager bench A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_graph.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_graph_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r4_graph_tests.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/r4_graph_ab.log
for rep in 1 2; do
for cfg in "--batch_size 32" "--model bert-large-uncased --seq_len 512 --batch_size 8" "--batch_size 128"; do
  for g in "" "--hip_graph"; do
    timeout -k 10 200 python bench.py --steps 30 --warmup 5 $cfg $g > gpurun_out/gp_bench.log 2>&1 || { tail -20 gpurun_out/gp_bench.log; exit 1; }
    echo "$cfg $g : $(tail -1 gpurun_out/gp_bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a gpurun_out/r4_graph_ab.log
  done
done
done
