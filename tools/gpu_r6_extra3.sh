# fp8 fragment chunk order (conflict-free frag8): fp8 numerics, MLM fp8 vs bf16 on one box, fp8 GEMM PMC again;
# segmented vs concatenated fp32 split-product GEMMs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 200 python tools/seg_vs_cat.py > gpurun_out/seg_vs_cat.log 2>&1 || { tail -20 gpurun_out/seg_vs_cat.log; exit 1; }
cat gpurun_out/seg_vs_cat.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fp8.py > gpurun_out/fp8_tests_r6c.log 2>&1 || { tail -30 gpurun_out/fp8_tests_r6c.log; exit 1; }
tail -2 gpurun_out/fp8_tests_r6c.log
: > gpurun_out/mlm_r6c.log
for dt in fp8 bf16 fp8; do
  timeout -k 10 400 python bench.py --steps 8 --warmup 3 --model roberta-large --task masked-lm --seq_len 512 --batch_size 64 --dtype $dt > gpurun_out/mlm_$dt.json 2>gpurun_out/mlm_$dt.err || { tail -20 gpurun_out/mlm_$dt.err; exit 1; }
  tail -1 gpurun_out/mlm_$dt.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('roberta-large MLM B=64 $dt', d['value'], d['ms_per_step'])" | tee -a gpurun_out/mlm_r6c.log || exit 1
done
PMC8=1 bash tools/gpu_r6_prof.sh
