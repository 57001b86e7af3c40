# fp8: dqkv / LN-backward dy q8_only on top of the FFN twins: fp8 GPU tests + same-box MLM fp8 A/B (hip._Q8_ONLY)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fp8.py > gpurun_out/tests_q8b.log 2>&1 || { tail -30 gpurun_out/tests_q8b.log; exit 1; }
tail -2 gpurun_out/tests_q8b.log
A="--steps 8 --warmup 3 --model roberta-large --task masked-lm --seq_len 512 --batch_size 64 --dtype fp8"
: > gpurun_out/q8b_ab.log
for v in True False True False; do
  timeout -k 10 300 python tools/bench_with.py ops.hip._Q8_ONLY=$v -- $A > gpurun_out/q8o.json 2>gpurun_out/q8o.err || { tail -20 gpurun_out/q8o.err; exit 1; }
  tail -1 gpurun_out/q8o.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('q8_only=$v roberta-large MLM B=64 fp8', d['value'], d['ms_per_step'])" | tee -a gpurun_out/q8b_ab.log || exit 1
done
timeout -k 10 300 python tools/fp8_quant_sites.py > gpurun_out/fp8_quant_sites.log 2>&1 || { tail -20 gpurun_out/fp8_quant_sites.log; exit 1; }
cat gpurun_out/fp8_quant_sites.log
bash tools/gpu_r6_tl_head.sh
