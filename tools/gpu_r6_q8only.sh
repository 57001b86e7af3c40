# fp8 FFN epilogues without the bf16 twins of their fp8 copies (hip._Q8_ONLY) and the gradient zeroing moved into Adam
# (Trainer.zero_grad_in_optimizer): GPU tests, same-box A/Bs, kernel statistics of the fp8 MLM step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fp8.py tests/test_gpu_e2e.py -k "fp8 or optimizer or adam" tests/test_gpu_ops.py > gpurun_out/tests_q8only.log 2>&1 || { tail -30 gpurun_out/tests_q8only.log; exit 1; }
tail -2 gpurun_out/tests_q8only.log
A="--steps 8 --warmup 3 --model roberta-large --task masked-lm --seq_len 512 --batch_size 64 --dtype fp8"
: > gpurun_out/q8only_ab.log
for v in True False True False; do
  timeout -k 10 300 python tools/bench_with.py ops.hip._Q8_ONLY=$v -- $A > gpurun_out/q8o.json 2>gpurun_out/q8o.err || { tail -20 gpurun_out/q8o.err; exit 1; }
  tail -1 gpurun_out/q8o.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('q8_only=$v roberta-large MLM B=64 fp8', d['value'], d['ms_per_step'])" | tee -a gpurun_out/q8only_ab.log || exit 1
done
: > gpurun_out/zg_ab.log
for v in True False True False; do
  for cfg in "--model bert-large-uncased --seq_len 512 --batch_size 8 --steps 30 --warmup 5" "--steps 10 --warmup 3"; do
    timeout -k 10 300 python tools/bench_with.py train.trainer.Trainer.zero_grad_in_optimizer=$v -- $cfg > gpurun_out/zg.json 2>gpurun_out/zg.err || { tail -20 gpurun_out/zg.err; exit 1; }
    tail -1 gpurun_out/zg.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('zero_in_adam=$v $cfg', d['value'], d['ms_per_step'])" | tee -a gpurun_out/zg_ab.log || exit 1
  done
done
PTAG=mlm_fp8_r6s PROF_ARGS="$A" bash tools/gpu_r6_prof.sh
