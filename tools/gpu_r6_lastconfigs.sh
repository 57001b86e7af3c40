# the README table's configs at the final HEAD, one box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
: > gpurun_out/configs_r6last.log
for cfg in "--steps 20 --warmup 5" \
           "--model bert-large-uncased --seq_len 512 --batch_size 8 --steps 30 --warmup 5" \
           "--model bert-large-uncased --seq_len 512 --batch_size 8 --steps 10 --warmup 3 --dtype fp32" \
           "--model bert-large-uncased --seq_len 512 --batch_size 64 --steps 8 --warmup 3" \
           "--steps 8 --warmup 3 --model roberta-large --task masked-lm --seq_len 512 --batch_size 64 --dtype fp8" \
           "--steps 8 --warmup 3 --model roberta-large --task masked-lm --seq_len 512 --batch_size 64 --dtype bf16" \
           "--batch_size 32 --steps 50 --warmup 10"; do
  timeout -k 10 300 python bench.py $cfg > gpurun_out/cfg.json 2>gpurun_out/cfg.err || { tail -20 gpurun_out/cfg.err; exit 1; }
  tail -1 gpurun_out/cfg.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg', d['value'], d['ms_per_step'], d['dtype'])" | tee -a gpurun_out/configs_r6last.log || exit 1
done
