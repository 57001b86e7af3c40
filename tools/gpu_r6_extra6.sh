# bf16 bert-large B=8 kernel trace for tools/timeline.py (critical path / overlap of the side streams)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/tl_bl8
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl_bl8 -o run -- python bench.py --model bert-large-uncased --seq_len 512 --batch_size 8 --steps 6 --warmup 3 > gpurun_out/tl_bl8.log 2>&1 || { tail -20 gpurun_out/tl_bl8.log; exit 1; }
f=$(find gpurun_out/tl_bl8 -name "*kernel_trace.csv" | head -1)
cp "$f" gpurun_out/trace_bl8_r6.csv
rm -rf gpurun_out/tl_bl8
head -2 gpurun_out/trace_bl8_r6.csv | cut -c1-400
python tools/timeline.py gpurun_out/trace_bl8_r6.csv --steps 4
