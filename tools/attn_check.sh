#!/bin/bash
# Attention-focused GPU check: build, attention tests, bert-large S=512 bench + kernel stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
python -m huggingface_sagemaker_tensorflow_distributed_amd._build > gpurun_out/build.log 2>&1 || { tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 600 python -m pytest tests/test_gpu_ops.py -x -q -m gpu -k "attention or fused_blocks" > gpurun_out/attn_tests.log 2>&1
rc=$?; tail -15 gpurun_out/attn_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --model bert-large-uncased --seq_len 512 --batch_size ${BATCH:-64} > gpurun_out/bench_large.log 2>&1 || { tail -20 gpurun_out/bench_large.log; exit 1; }
tail -1 gpurun_out/bench_large.log
rm -rf gpurun_out/prof_large
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_large -o run -- python bench.py --steps 5 --warmup 3 --model bert-large-uncased --seq_len 512 --batch_size ${BATCH:-64} > gpurun_out/prof_large.log 2>&1 || { tail -20 gpurun_out/prof_large.log; exit 1; }
find gpurun_out/prof_large -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/kernel_stats_large.csv
head -25 gpurun_out/kernel_stats_large.csv | cut -d, -f1-5 | cut -c1-160
