#!/bin/bash
# Round-3 A/B: graph tests, roberta-large MLM bf16 vs fp8 (fused LN quantisation), bert-large B=8 eager vs
# whole-step HIP graph, bert-base B=32 eager vs graph. One line per run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_graph.py -x -q --timeout 120 --timeout-method thread > gpurun_out/graph_tests.log 2>&1
rc=$?; tail -3 gpurun_out/graph_tests.log; [ $rc -eq 0 ] || exit $rc
run() {
  echo -n "$* : "
  timeout -k 10 300 python bench.py "$@" 2>gpurun_out/ab_err.log | grep metric | \
    python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])' || { tail -5 gpurun_out/ab_err.log; exit 1; }
}
M="--model roberta-large --task masked-lm --seq_len 512 --batch_size 64 --steps 10 --warmup 3"
run $M --dtype bf16 && run $M --dtype fp8 && run $M --dtype bf16 && run $M --dtype fp8 || exit 1
L="--model bert-large-uncased --seq_len 512 --batch_size 8 --steps 30 --warmup 5"
run $L && run $L --hip_graph && run $L && run $L --hip_graph || exit 1
S="--batch_size 32 --steps 30 --warmup 5"
run $S && run $S --hip_graph || exit 1
