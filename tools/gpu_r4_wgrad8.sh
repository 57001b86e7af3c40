#!/bin/bash
# fp8 TT weight gradient: tr8 lane-mapping probe, numerics tests, kernel A/B vs bf16, roberta-large MLM fp8 vs bf16
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 ./tools/experiments/tr8_probe > gpurun_out/tr8_probe.log 2>&1 && cat gpurun_out/tr8_probe.log | tail -3 &&
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_fp8.py \
  -k "wgrad or fused_ln_quant_in_the_step or mlm_step" > gpurun_out/wgrad8_tests.log 2>&1 && tail -3 gpurun_out/wgrad8_tests.log &&
timeout -k 10 200 python -u tools/wgrad8_ab.py 20 > gpurun_out/wgrad8_ab.jsonl 2>&1 && cat gpurun_out/wgrad8_ab.jsonl
