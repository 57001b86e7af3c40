# (historical A/B: hip._WGRAD_ATOMIC was removed after it)
# side-stream bf16 weight gradients: K-split slabs + reduce pass (default) vs fp32 atomics into the gradient
# (hip._WGRAD_ATOMIC), headline and bert-large B=64
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
: > gpurun_out/atomic_ab.log
for r in 1 2; do
  for v in False True; do
    for cfg in "--steps 10 --warmup 3" "--model bert-large-uncased --seq_len 512 --batch_size 64 --steps 8 --warmup 3"; do
      timeout -k 10 300 python tools/bench_with.py ops.hip._WGRAD_ATOMIC=$v -- $cfg > gpurun_out/at.json 2>gpurun_out/at.err || { tail -20 gpurun_out/at.err; exit 1; }
      tail -1 gpurun_out/at.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('wgrad_atomic=$v $cfg', d['value'], d['ms_per_step'])" | tee -a gpurun_out/atomic_ab.log || exit 1
    done
  done
done
