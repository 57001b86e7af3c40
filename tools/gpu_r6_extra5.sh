# seg GEMM operand-placement probe; bf16 bert-large B=8 bench + kernel statistics
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 200 python tools/seg_vs_cat.py > gpurun_out/seg_vs_cat.log 2>&1 || { tail -20 gpurun_out/seg_vs_cat.log; exit 1; }
cat gpurun_out/seg_vs_cat.log
timeout -k 10 300 python bench.py --model bert-large-uncased --seq_len 512 --batch_size 8 --steps 30 --warmup 5 > gpurun_out/bench_bl8_r6i.log 2>&1 || { tail -20 gpurun_out/bench_bl8_r6i.log; exit 1; }
tail -1 gpurun_out/bench_bl8_r6i.log | cut -c1-200
PTAG=bl8_r6i PROF_ARGS="--model bert-large-uncased --seq_len 512 --batch_size 8 --steps 10 --warmup 3" bash tools/gpu_r6_prof.sh
