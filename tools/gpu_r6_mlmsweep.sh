# roberta-large MLM fp8 (and bert-large B=64) knobs at HEAD: Adam slice size (HSD_OPT_BUCKET_MB)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
: > gpurun_out/mlmsweep.log
for r in 1 2; do
  for e in "X=0" "HSD_OPT_BUCKET_MB=8" "HSD_OPT_BUCKET_MB=32" "HSD_OPT_BUCKET_MB=64"; do
    for cfg in "--steps 8 --warmup 3 --model roberta-large --task masked-lm --seq_len 512 --batch_size 64 --dtype fp8" "--model bert-large-uncased --seq_len 512 --batch_size 64 --steps 8 --warmup 3"; do
      env $e timeout -k 10 300 python bench.py $cfg > gpurun_out/ms.json 2>gpurun_out/ms.err || { tail -20 gpurun_out/ms.err; exit 1; }
      tail -1 gpurun_out/ms.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$e $cfg', d['value'], d['ms_per_step'])" | tee -a gpurun_out/mlmsweep.log || exit 1
    done
  done
done
