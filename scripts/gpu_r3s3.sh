mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3s3_suite2.log 2>&1 || exit 1
for b in 2048 1536; do timeout -k 10 200 python -u bench.py --steps 15 --warmup 4 --batch_size $b >> gpurun_out/r3s3_batch.log 2>&1 || exit 1; done
timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --model bert-large-uncased --seq_len 512 --batch_size 8 >> gpurun_out/r3s3_batch.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3s3_prof2 -o run -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/r3s3_prof2.log 2>&1 || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3s3_prof_b8 -o run -- python3 bench.py --steps 20 --warmup 5 --model bert-large-uncased --seq_len 512 --batch_size 8 > gpurun_out/r3s3_prof_b8.log 2>&1
