#!/bin/bash
# Round 5, first GPU pass after the dropout-mask redesign and the captured-DP ordering fix:
# (1) attention kernel timings p = 0 / 0.1 (S = 128 headline shape; S = 512 bert-large B = 64 shape, keep bits on/off)
# (2) the delayed-side-stream ordering test without the engine's capture edge (expected to FAIL), then the GPU tier
# (3) headline bench, bert-large S=512 B=8 with the small-step wgrad plan on (default) / off
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
{
  timeout -k 10 120 python tools/attn_one.py 0.1 20 &&
  ATTN_SHAPE=64,512,16 timeout -k 10 120 python tools/attn_one.py 0.1 20 &&
  ATTN_KMASK=0 ATTN_SHAPE=64,512,16 timeout -k 10 120 python tools/attn_one.py 0.1 20
} > gpurun_out/attn_r5a.log 2>&1 || { echo "attn timing failed"; tail -20 gpurun_out/attn_r5a.log; exit 1; }
cat gpurun_out/attn_r5a.log
HSD_ENGINE_CAPTURE_DEPS=0 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_comm.py -k delayed_wgrad > gpurun_out/race_nofix.log 2>&1
echo "without the capture edge: exit $? (expected 1)"; grep -E "passed|failed|assert" gpurun_out/race_nofix.log | tail -3
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -15 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | cut -c1-200
: > gpurun_out/mingrid_r5.log
for r in 1 2; do
  for g in 0 192; do
    HSD_WGRAD_MIN_GRID=$g timeout -k 10 300 python bench.py --model bert-large-uncased --seq_len 512 --batch_size 8 --steps 30 --warmup 5 2>/dev/null | tail -1 | cut -c1-120 | sed "s/^/bl8 min_grid=$g /" >> gpurun_out/mingrid_r5.log || exit 1
  done
done
cat gpurun_out/mingrid_r5.log
