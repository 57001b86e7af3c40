# bench of the secondary BASELINE.json configs (bert-large S=512, roberta-large MLM S=512 bf16 / fp8), one GPU
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --model bert-large-uncased --seq_len 512 --batch_size 64 > gpurun_out/big_bertlarge.log 2>&1 || { tail -20 gpurun_out/big_bertlarge.log; exit 1; }
tail -1 gpurun_out/big_bertlarge.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --model roberta-large --task masked-lm --seq_len 512 --batch_size 64 > gpurun_out/big_roberta_bf16.log 2>&1 || { tail -20 gpurun_out/big_roberta_bf16.log; exit 1; }
tail -1 gpurun_out/big_roberta_bf16.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --model roberta-large --task masked-lm --seq_len 512 --batch_size 64 --dtype fp8 > gpurun_out/big_roberta_fp8.log 2>&1 || { tail -20 gpurun_out/big_roberta_fp8.log; exit 1; }
tail -1 gpurun_out/big_roberta_fp8.log
