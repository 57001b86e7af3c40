# host issue cost of the bert-large B=8 step (is the eager step host-bound?) + baseline benches on this box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python tools/host_profile.py > gpurun_out/host_bl8.log 2>&1 || { tail -20 gpurun_out/host_bl8.log; exit 1; }
head -60 gpurun_out/host_bl8.log
timeout -k 10 300 python bench.py --model bert-large-uncased --seq_len 512 --batch_size 8 --steps 30 --warmup 5 > gpurun_out/bench_bl8.log 2>&1 || { tail -20 gpurun_out/bench_bl8.log; exit 1; }
tail -1 gpurun_out/bench_bl8.log | cut -c1-200
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_head.log 2>&1 || { tail -20 gpurun_out/bench_head.log; exit 1; }
tail -1 gpurun_out/bench_head.log | cut -c1-200
