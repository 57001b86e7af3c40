# (historical A/B: the CU-masked side stream was measured 18-47 % slower and removed)
# weight-gradient side stream restricted to part of the CUs (hip._SIDE_CU_FRACTION: 0 = all, 0.5, 0.75): headline,
# bert-large B=8, roberta-large MLM fp8
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
: > gpurun_out/cumask_ab.log
for r in 1 2; do
  for f in 0 0.75 0.5; do
    for cfg in "--steps 10 --warmup 3" "--model bert-large-uncased --seq_len 512 --batch_size 8 --steps 30 --warmup 5" "--steps 8 --warmup 3 --model roberta-large --task masked-lm --seq_len 512 --batch_size 64 --dtype fp8"; do
      timeout -k 10 300 python tools/bench_with.py ops.hip._SIDE_CU_FRACTION=$f -- $cfg > gpurun_out/cm.json 2>gpurun_out/cm.err || { tail -20 gpurun_out/cm.err; exit 1; }
      tail -1 gpurun_out/cm.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('side_cu_fraction=$f $cfg', d['value'], d['ms_per_step'])" | tee -a gpurun_out/cumask_ab.log || exit 1
    done
  done
done
