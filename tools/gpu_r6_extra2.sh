# fp32 bench + kernel stats after the SEG-pointer fix, then the fp8 GEMM PMC passes
timeout -k 10 300 python bench.py --model bert-large-uncased --seq_len 512 --batch_size 8 --dtype fp32 --steps 20 --warmup 5 > gpurun_out/bench_fp32_bl8_r6b.log 2>&1 || { tail -20 gpurun_out/bench_fp32_bl8_r6b.log; exit 1; }
tail -1 gpurun_out/bench_fp32_bl8_r6b.log | cut -c1-160
PTAG=fp32_bl8_r6b PROF_ARGS="--model bert-large-uncased --seq_len 512 --batch_size 8 --dtype fp32 --steps 8 --warmup 3" bash tools/gpu_r6_prof.sh || exit 1
PMC8=1 bash tools/gpu_r6_prof.sh
