# MLM head weight gradients (the tied decoder's [50,432 x 1,024] over the masked tokens, < 8,192 of them): the small-step
# 128 x 128 plan (default) vs the cost model's tiles (HSD_G2_SMALL_TT=0 forces 256 x 256; under --dtype fp8 the encoder's
# weight gradients are fp8 and unaffected)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
: > gpurun_out/headtt.log
for r in 1 2 3; do
  for e in "X=0" "HSD_G2_SMALL_TT=0"; do
    cfg="--steps 8 --warmup 3 --model roberta-large --task masked-lm --seq_len 512 --batch_size 64 --dtype fp8"
    env $e timeout -k 10 300 python bench.py $cfg > gpurun_out/ht.json 2>gpurun_out/ht.err || { tail -20 gpurun_out/ht.err; exit 1; }
    tail -1 gpurun_out/ht.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$e MLM fp8', d['value'], d['ms_per_step'])" | tee -a gpurun_out/headtt.log || exit 1
  done
done
