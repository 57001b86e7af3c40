#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
python -m huggingface_sagemaker_tensorflow_distributed_amd._build > gpurun_out/build.log 2>&1 || { tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 600 python -m pytest tests/test_gpu_fp8.py -x -q -m gpu > gpurun_out/fp8_tests.log 2>&1
rc=$?; tail -5 gpurun_out/fp8_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 8 --warmup 3 --model roberta-large --task masked-lm --seq_len 512 --batch_size ${BATCH:-64} --dtype fp8 > gpurun_out/bench_rl_fp8.log 2>&1 || { tail -20 gpurun_out/bench_rl_fp8.log; exit 1; }
tail -1 gpurun_out/bench_rl_fp8.log
rm -rf gpurun_out/prof_fp8
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_fp8 -o run -- python bench.py --steps 4 --warmup 2 --model roberta-large --task masked-lm --seq_len 512 --batch_size ${BATCH:-64} --dtype fp8 > gpurun_out/prof_fp8.log 2>&1 || { tail -20 gpurun_out/prof_fp8.log; exit 1; }
find gpurun_out/prof_fp8 -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/kernel_stats_fp8.csv
