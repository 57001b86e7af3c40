#!/bin/bash
# HIP graph check: build, graph + dropout-sensitive tests, bench eager vs graph at small and large batch.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
python -m huggingface_sagemaker_tensorflow_distributed_amd._build > gpurun_out/build.log 2>&1 || { tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 600 python -m pytest tests/test_gpu_graph.py tests/test_gpu_ops.py tests/test_gpu_e2e.py -x -q -m gpu > gpurun_out/graph_tests.log 2>&1
rc=$?; tail -5 gpurun_out/graph_tests.log
[ $rc -eq 0 ] || exit $rc
for B in 32 256 1024; do
  for G in "" "--hip_graph"; do
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --batch_size $B $G > gpurun_out/bench_g.log 2>&1 || { tail -20 gpurun_out/bench_g.log; exit 1; }
    echo "B=$B $G $(tail -1 gpurun_out/bench_g.log | cut -c1-140)"
  done
done
