#!/bin/bash
# The reference's whole job on one MI355X: `python launch.py` at its literal hyperparameters
# (launch.py:14-17: bert-large-uncased-whole-word-masking, epochs 1, per-rank batch 8, eval batch 2, S = 512) over
# IMDB-sized synthetic splits (25,000 train / 25,000 test), in bf16 and fp32; logs train_runtime and the evaluation's
# wall time / seq/s. Optional: BENCH=1 runs the headline bench first; DTYPES overrides "bf16 fp32".
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r6}
if [ -n "$BENCH" ]; then
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_${TAG}.log 2>&1 || { tail -20 gpurun_out/bench_${TAG}.log; exit 1; }
  tail -1 gpurun_out/bench_${TAG}.log
fi
# MODES (default "job"): job = train + evaluate at the defaults; eval = the evaluation alone at the defaults;
# eval_b2 = the evaluation alone, one forward per batch of 2 (no coalescing), replayed graphs; eval_eager = the same,
# eager forwards (the "before"). EAGER=1 adds eval_eager.
for dt in ${DTYPES:-bf16 fp32}; do
  for mode in ${MODES:-job} ${EAGER:+eval_eager}; do
    rm -rf output
    case $mode in
      job) extra="HSD_DO_TRAIN=True" ;;
      eval) extra="HSD_DO_TRAIN=False" ;;
      eval_b2) extra="HSD_DO_TRAIN=False HSD_EVAL_COALESCE_TOKENS=0" ;;
      eval_eager) extra="HSD_DO_TRAIN=False HSD_EVAL_HIP_GRAPH=False HSD_EVAL_COALESCE_TOKENS=0" ;;
    esac
    env $extra HSD_DTYPE=$dt HSD_MAX_STEPS=0 HSD_NUM_TRAIN=${NTRAIN:-25000} HSD_NUM_EVAL=${NEVAL:-25000} \
      timeout -k 10 ${JOB_TIMEOUT:-600} python -u launch.py > gpurun_out/${mode}_${TAG}_${dt}.log 2>&1
    rc=$?
    grep -E "train_runtime =|eval_runtime =|Epoch 1/1|loss = |accuracy = " gpurun_out/${mode}_${TAG}_${dt}.log | tail -8
    [ $rc -eq 0 ] || { tail -30 gpurun_out/${mode}_${TAG}_${dt}.log; exit $rc; }
  done
done
