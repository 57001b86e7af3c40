timeout -k 10 300 python bench.py --model bert-large-uncased --seq_len 512 --batch_size 8 --dtype fp32 --steps 20 --warmup 5 > gpurun_out/bench_fp32_bl8_r6a.log 2>&1 || { tail -20 gpurun_out/bench_fp32_bl8_r6a.log; exit 1; }
tail -1 gpurun_out/bench_fp32_bl8_r6a.log | cut -c1-160
timeout -k 10 300 python bench.py --model bert-large-uncased --seq_len 512 --batch_size 8 --steps 30 --warmup 5 > gpurun_out/bench_bl8_r6a.log 2>&1 || { tail -20 gpurun_out/bench_bl8_r6a.log; exit 1; }
tail -1 gpurun_out/bench_bl8_r6a.log | cut -c1-160
TAG=r6a MODES=eval DTYPES="bf16 fp32" bash tools/gpu_r6_job.sh
