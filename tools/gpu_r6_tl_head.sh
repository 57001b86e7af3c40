# headline (bert-base S=128 B=1024) and bert-large B=8 kernel traces for tools/timeline.py (idle gaps, exposed kernels)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for tag in head bl8; do
  if [ $tag = head ]; then A="--steps 4 --warmup 3"; else A="--model bert-large-uncased --seq_len 512 --batch_size 8 --steps 6 --warmup 3"; fi
  rm -rf gpurun_out/tl_$tag
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl_$tag -o run -- python bench.py $A > gpurun_out/tl_$tag.log 2>&1 || { tail -20 gpurun_out/tl_$tag.log; exit 1; }
  f=$(find gpurun_out/tl_$tag -name "*kernel_trace.csv" | head -1)
  cp "$f" gpurun_out/trace_${tag}_r6.csv
  rm -rf gpurun_out/tl_$tag
  python tools/timeline.py gpurun_out/trace_${tag}_r6.csv --steps 3 > gpurun_out/timeline_${tag}_r6.txt || exit 1
  head -40 gpurun_out/timeline_${tag}_r6.txt
done
