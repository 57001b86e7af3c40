# HEAD: the reference's whole job in bf16 and fp32 (train_runtime, eval seconds / seq/s with coalesced, graph-replayed
# evaluation), then kernel statistics of the headline, bert-large B=8 and the fp8 MLM step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=r6head bash tools/gpu_r6_job.sh || exit 1
PTAG=head_r6 PROF_ARGS="--steps 10 --warmup 3" bash tools/gpu_r6_prof.sh || exit 1
PTAG=bl8_r6 PROF_ARGS="--model bert-large-uncased --seq_len 512 --batch_size 8 --steps 20 --warmup 5" bash tools/gpu_r6_prof.sh || exit 1
PTAG=mlm_fp8_r6h PROF_ARGS="--steps 6 --warmup 3 --model roberta-large --task masked-lm --seq_len 512 --batch_size 64 --dtype fp8" bash tools/gpu_r6_prof.sh || exit 1
