# (historical A/B: the switches it sets, hip._WGRAD8_SPLITS / hip._WGRAD_SPLIT_DIV, were replaced by the measured rule hip._WGRAD8_SIDE_SPLITS)
# side-stream weight-gradient K-splits: bf16 headline (hip._WGRAD_SPLIT_DIV: the cost model's splits / n) and fp8 MLM
# (hip._WGRAD8_SPLITS: 0 model, n fixed, -n model / n)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
: > gpurun_out/wsplit_ab.log
for r in 1 2; do
  for d in 1 2 4; do
    timeout -k 10 300 python tools/bench_with.py ops.hip._WGRAD_SPLIT_DIV=$d -- --steps 10 --warmup 3 > gpurun_out/ws.json 2>gpurun_out/ws.err || { tail -20 gpurun_out/ws.err; exit 1; }
    tail -1 gpurun_out/ws.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('wgrad_split_div=$d headline', d['value'], d['ms_per_step'])" | tee -a gpurun_out/wsplit_ab.log || exit 1
  done
  for sp in 0 2 3 -2; do
    timeout -k 10 300 python tools/bench_with.py ops.hip._WGRAD8_SPLITS=$sp -- --steps 8 --warmup 3 --model roberta-large --task masked-lm --seq_len 512 --batch_size 64 --dtype fp8 > gpurun_out/w8.json 2>gpurun_out/w8.err || { tail -20 gpurun_out/w8.err; exit 1; }
    tail -1 gpurun_out/w8.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('wgrad8_splits=$sp roberta-large MLM B=64 fp8', d['value'], d['ms_per_step'])" | tee -a gpurun_out/wsplit_ab.log || exit 1
  done
done
for d in 1 2; do
  timeout -k 10 300 python tools/bench_with.py ops.hip._WGRAD_SPLIT_DIV=$d -- --model bert-large-uncased --seq_len 512 --batch_size 64 --steps 8 --warmup 3 > gpurun_out/ws.json 2>gpurun_out/ws.err || { tail -20 gpurun_out/ws.err; exit 1; }
  tail -1 gpurun_out/ws.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('wgrad_split_div=$d bert-large B=64', d['value'], d['ms_per_step'])" | tee -a gpurun_out/wsplit_ab.log || exit 1
done
