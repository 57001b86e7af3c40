#!/bin/bash
# Round 5 pass L: out-projection dgrad writing the streaming attention backward's delta rows (E2_STORE_RDOT)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_ops.py -k "row_dot or fused_blocks or attention or persistent or splitk" -x -q --timeout 300 --timeout-method thread > gpurun_out/rdot_tests.log 2>&1
rc=$?; tail -3 gpurun_out/rdot_tests.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/rdot_ab.log
for v in 0 1 0 1; do
  HSD_ATTN_DELTA_EPI=$v timeout -k 10 300 python bench.py --model bert-large-uncased --seq_len 512 --batch_size 8 --steps 30 --warmup 5 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bert-large B=8 DELTA_EPI=$v', d['value'], d['ms_per_step'])" | tee -a gpurun_out/rdot_ab.log || exit 1
done
for v in 0 1; do
  HSD_ATTN_DELTA_EPI=$v timeout -k 10 300 python bench.py --model bert-large-uncased --seq_len 512 --batch_size 64 --steps 8 --warmup 3 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bert-large B=64 DELTA_EPI=$v', d['value'], d['ms_per_step'])" | tee -a gpurun_out/rdot_ab.log || exit 1
done
