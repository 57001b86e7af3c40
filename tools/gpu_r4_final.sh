#!/bin/bash
# Round-4 HEAD evidence: full GPU tier, smoke, headline bench x2 + kernel stats, the reference's per-rank config and
# the fp8 config (each step time-limited, chained).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_gpu_suite.log 2>&1
rc=$?; tail -4 gpurun_out/r4_gpu_suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4_smoke.log 2>&1 || { tail -20 gpurun_out/r4_smoke.log; exit 1; }
tail -1 gpurun_out/r4_smoke.log
for i in 1 2; do
  timeout -k 10 300 python bench.py > gpurun_out/r4_bench_$i.log 2>&1 || { tail -20 gpurun_out/r4_bench_$i.log; exit 1; }
  tail -1 gpurun_out/r4_bench_$i.log | cut -c1-220
done
timeout -k 10 300 python bench.py --model bert-large-uncased --seq_len 512 --batch_size 8 --steps 30 --warmup 5 > gpurun_out/r4_bench_bl8.log 2>&1 || exit 1
tail -1 gpurun_out/r4_bench_bl8.log | cut -c1-220
timeout -k 10 300 python bench.py --model roberta-large --task masked-lm --seq_len 512 --batch_size 64 --dtype fp8 > gpurun_out/r4_bench_fp8.log 2>&1 || exit 1
tail -1 gpurun_out/r4_bench_fp8.log | cut -c1-220
timeout -k 10 300 python bench.py --model roberta-large --task masked-lm --seq_len 512 --batch_size 64 --dtype bf16 > gpurun_out/r4_bench_mlm_bf16.log 2>&1 || exit 1
tail -1 gpurun_out/r4_bench_mlm_bf16.log | cut -c1-220
PROF_NAME=r4_head bash tools/prof_r4.sh --steps 8 --warmup 3
