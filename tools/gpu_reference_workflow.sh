#!/bin/bash
# The reference's own workflow on one MI355X, end to end:
#   1. `python launch.py` exactly as the reference ships it (bert-large-uncased-whole-word-masking, per-rank batch 8,
#      eval batch 2, seq 512, one epoch capped at 20 steps; synthetic data / random-init weights: offline box),
#   2. `scripts/singe_node_train.py` (MirroredStrategy semantics) on bert-base,
#   3. the saved checkpoint loaded by HF transformers (AutoModelForSequenceClassification.from_pretrained) and its
#      logits compared with this framework's HIP forward on the same batch.
# Writes its logs and results under gpurun_out/refwf/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/refwf
rm -rf "$OUT"
mkdir -p "$OUT"
rm -rf output/hf-tf-bert-1node-mi355x-*
timeout -k 10 400 python launch.py > $OUT/launch.log 2>&1 || { tail -30 $OUT/launch.log; exit 1; }
grep -E "train_runtime|Train results|Eval results| = " $OUT/launch.log | tail -12
# the estimator writes per-job dirs like SageMaker's /opt/ml/{model,output/data}: output/<job name>/{model,data}
cp -r output/hf-tf-bert-1node-mi355x-*/ $OUT/launch && ls -R $OUT/launch
timeout -k 10 400 python scripts/singe_node_train.py --model_name_or_path bert-base-uncased --epochs 1 \
  --train_batch_size 64 --eval_batch_size 64 --max_seq_length 128 --max_steps 30 --num_train_examples 4096 \
  --num_eval_examples 512 --output_data_dir $OUT/single/data --model_dir $OUT/single/model > $OUT/single.log 2>&1 \
  || { tail -30 $OUT/single.log; exit 1; }
grep -E " = " $OUT/single.log | tail -6
timeout -k 10 300 python tools/hf_load_check.py $OUT/single/model > $OUT/hf_load.log 2>&1 || { tail -30 $OUT/hf_load.log; exit 1; }
tail -3 $OUT/hf_load.log
find $OUT -name "*.safetensors" -delete
