# (historical A/B: hip._WGRAD8_SIDE_WGS was removed after it; the fixed 2 splits stayed)
# side-stream fp8 weight gradients: fixed 2 token splits vs splits for ~64 / 128 / 192 workgroups per GEMM
# (hip._WGRAD8_SIDE_WGS), roberta-large MLM fp8
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
: > gpurun_out/w8wgs_ab.log
for r in 1 2; do
  for w in 0 64 128 192; do
    timeout -k 10 300 python tools/bench_with.py ops.hip._WGRAD8_SIDE_WGS=$w -- --steps 8 --warmup 3 --model roberta-large --task masked-lm --seq_len 512 --batch_size 64 --dtype fp8 > gpurun_out/w8.json 2>gpurun_out/w8.err || { tail -20 gpurun_out/w8.err; exit 1; }
    tail -1 gpurun_out/w8.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('wgrad8_side_wgs=$w roberta-large MLM B=64 fp8', d['value'], d['ms_per_step'])" | tee -a gpurun_out/w8wgs_ab.log || exit 1
  done
done
