# segmented-K fp32 GEMMs without the LDS-promoted segment pointers: seg vs concatenated, fp32 tests, fp32 bench B=8
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 200 python tools/seg_vs_cat.py > gpurun_out/seg_vs_cat.log 2>&1 || { tail -20 gpurun_out/seg_vs_cat.log; exit 1; }
cat gpurun_out/seg_vs_cat.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fp32.py > gpurun_out/fp32_tests_r6h.log 2>&1 || { tail -30 gpurun_out/fp32_tests_r6h.log; exit 1; }
tail -2 gpurun_out/fp32_tests_r6h.log
timeout -k 10 300 python bench.py --model bert-large-uncased --seq_len 512 --batch_size 8 --dtype fp32 --steps 20 --warmup 5 > gpurun_out/bench_fp32_bl8_r6h.log 2>&1 || { tail -20 gpurun_out/bench_fp32_bl8_r6h.log; exit 1; }
tail -1 gpurun_out/bench_fp32_bl8_r6h.log | cut -c1-200
PTAG=fp32_bl8_r6h PROF_ARGS="--model bert-large-uncased --seq_len 512 --batch_size 8 --dtype fp32 --steps 8 --warmup 3" bash tools/gpu_r6_prof.sh
