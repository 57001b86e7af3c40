# Two DP ranks sharing the one GPU of a gpurun box (gloo transport: RCCL refuses two ranks on one device):
# exercises the world>1 GPU training path (bucket hooks from the HIP backward, async all-reduce, max-over-ranks
# timing) end to end. Not a performance number.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp HSD_DIST_BACKEND=gloo
mkdir -p gpurun_out
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --batch_size 64 > gpurun_out/two_ranks.log 2>&1 || { tail -30 gpurun_out/two_ranks.log; exit 1; }
grep '"metric"' gpurun_out/two_ranks.log
# MLM (decoder tied to the word embeddings: the tied-weight readiness case) on two ranks
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --steps 3 --warmup 2 --batch_size 16 --task masked-lm --model roberta-base > gpurun_out/two_ranks_mlm.log 2>&1 || { tail -30 gpurun_out/two_ranks_mlm.log; exit 1; }
grep '"metric"' gpurun_out/two_ranks_mlm.log | cut -c1-160
# the reference entry point (Horovod semantics) through the launcher: 2 ranks, bert-base, cross-rank sync check
timeout -k 10 400 python -m huggingface_sagemaker_tensorflow_distributed_amd.launcher --nproc-per-node 2 --output-data-dir gpurun_out/tr2/data --model-dir gpurun_out/tr2/model scripts/train.py --model_name_or_path bert-base-uncased --epochs 1 --train_batch_size 32 --eval_batch_size 32 --max_steps 20 --num_train_examples 1280 --num_eval_examples 128 --max_seq_length 128 --dtype bf16 --check_sync 5 --benchmark true > gpurun_out/two_ranks_train.log 2>&1 || { tail -30 gpurun_out/two_ranks_train.log; exit 1; }
grep -E "Epoch|eval|throughput" gpurun_out/two_ranks_train.log | tail -5
rm -f gpurun_out/tr2/model/*.safetensors
