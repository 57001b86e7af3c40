# weight-gradient grid target for small steps (HSD_WGRAD_MIN_GRID, K <= 8,192 tokens): bert-large B=8 and bert-base B=32
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
: > gpurun_out/bl8sweep2.log
for r in 1 2; do
  for g in 192 128 384 512 768; do
    for cfg in "--model bert-large-uncased --seq_len 512 --batch_size 8 --steps 30 --warmup 5" "--batch_size 32 --steps 30 --warmup 5"; do
      HSD_WGRAD_MIN_GRID=$g timeout -k 10 300 python bench.py $cfg > gpurun_out/sw.json 2>gpurun_out/sw.err || { tail -20 gpurun_out/sw.err; exit 1; }
      tail -1 gpurun_out/sw.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('HSD_WGRAD_MIN_GRID=$g $cfg', d['value'], d['ms_per_step'])" | tee -a gpurun_out/bl8sweep2.log || exit 1
    done
  done
done
