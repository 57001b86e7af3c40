#!/bin/bash
# streaming attention keep mask + fused fp8 embedding copy: tests, kernel timing, bench A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_fp8.py -x -q -m gpu --timeout 120 --timeout-method thread -k "attention or fused_blocks or attn or keep_mask or fp8 or q8 or embed" > gpurun_out/r4_s512_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4_s512_tests.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/r4_s512_attn.log
for km in 1 0 1 0; do for shp in 64,512,16 8,512,16; do
  echo "shape $shp kmask $km: $(ATTN_SHAPE=$shp ATTN_KMASK=$km timeout -k 10 120 python tools/attn_one.py 0.1 20 2>&1 | grep -v amdgpu | tail -1)" >> gpurun_out/r4_s512_attn.log || exit 1
done; done
cat gpurun_out/r4_s512_attn.log
: > gpurun_out/r4_s512_bench.log
for rep in 1 2; do for km in 1 0; do
  for cfg in "--model bert-large-uncased --seq_len 512 --batch_size 8" "--model roberta-large --task masked-lm --seq_len 512 --batch_size 64"; do
    HSD_ATTN_KMASK=$km timeout -k 10 300 python bench.py --steps 20 --warmup 5 $cfg > gpurun_out/s512_b.log 2>&1 || { tail -20 gpurun_out/s512_b.log; exit 1; }
    echo "$cfg KMASK=$km : $(tail -1 gpurun_out/s512_b.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a gpurun_out/r4_s512_bench.log
  done
done; done
