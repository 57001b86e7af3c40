#!/bin/bash
# Round 5 GPU pass B: comm tests (ordering fix + capture-safe engine teardown), the GPU tier, the headline bench,
# bert-large S=512 B=8 min-grid A/B, the dropout-off bound of the headline, the reference's literal fp32 config.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_comm.py > gpurun_out/comm_r5.log 2>&1
rc=$?; grep -E "PASSED|FAILED|passed|failed" gpurun_out/comm_r5.log | tail -10; [ $rc -eq 0 ] || exit $rc
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -5 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | cut -c1-200
python - <<'PY'
import json
from huggingface_sagemaker_tensorflow_distributed_amd.models import resolve_config
import os
os.makedirs("/tmp/bb_nodrop", exist_ok=True)
c = resolve_config("bert-base-uncased").replace(hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
json.dump(c.to_hf_dict() if hasattr(c, "to_hf_dict") else c.hf_dict(), open("/tmp/bb_nodrop/config.json", "w"))
PY
timeout -k 10 300 python bench.py --model /tmp/bb_nodrop --steps 20 --warmup 5 2>/dev/null | tail -1 | cut -c1-160 | sed "s/^/no-dropout bound: /" || echo "nodrop bench failed"
: > gpurun_out/mingrid_r5.log
for r in 1 2; do
  for g in 0 192; do
    HSD_WGRAD_MIN_GRID=$g timeout -k 10 300 python bench.py --model bert-large-uncased --seq_len 512 --batch_size 8 --steps 30 --warmup 5 2>/dev/null | tail -1 | cut -c1-120 | sed "s/^/bl8 min_grid=$g /" >> gpurun_out/mingrid_r5.log || exit 1
  done
done
cat gpurun_out/mingrid_r5.log
timeout -k 10 600 python bench.py --model bert-large-uncased --seq_len 512 --batch_size 8 --dtype fp32 --steps 10 --warmup 3 > gpurun_out/bench_fp32.log 2>&1 || { tail -20 gpurun_out/bench_fp32.log; exit 1; }
tail -1 gpurun_out/bench_fp32.log | cut -c1-250
