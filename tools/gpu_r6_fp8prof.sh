# kernel statistics of roberta-large MLM S=512 B=64 fp8 at HEAD (BASELINE config 5)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
PTAG=mlm_fp8_r6s PROF_ARGS="--steps 6 --warmup 3 --model roberta-large --task masked-lm --seq_len 512 --batch_size 64 --dtype fp8" bash tools/gpu_r6_prof.sh
