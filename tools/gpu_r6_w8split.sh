# (historical A/B: the switches it sets, hip._WGRAD8_SPLITS / hip._WGRAD_SPLIT_DIV, were replaced by the measured rule hip._WGRAD8_SIDE_SPLITS)
# fp8 weight-gradient token splits under the side-stream overlap (hip._WGRAD8_SPLITS: 0 = cost model) + MLM bf16 at HEAD
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
A="--steps 8 --warmup 3 --model roberta-large --task masked-lm --seq_len 512 --batch_size 64"
: > gpurun_out/w8split_ab.log
for r in 1 2; do
  for sp in 0 1 2 4; do
    timeout -k 10 300 python tools/bench_with.py ops.hip._WGRAD8_SPLITS=$sp -- $A --dtype fp8 > gpurun_out/w8.json 2>gpurun_out/w8.err || { tail -20 gpurun_out/w8.err; exit 1; }
    tail -1 gpurun_out/w8.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('wgrad8_splits=$sp roberta-large MLM B=64 fp8', d['value'], d['ms_per_step'])" | tee -a gpurun_out/w8split_ab.log || exit 1
  done
done
timeout -k 10 300 python bench.py $A --dtype bf16 > gpurun_out/mlm_bf16.json 2>gpurun_out/mlm_bf16.err || { tail -20 gpurun_out/mlm_bf16.err; exit 1; }
tail -1 gpurun_out/mlm_bf16.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('roberta-large MLM B=64 bf16', d['value'], d['ms_per_step'])" | tee -a gpurun_out/w8split_ab.log
