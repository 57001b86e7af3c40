# kernel-trace timelines at HEAD: roberta-large MLM fp8 and bert-large B=8 (tools/timeline.py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for tag in fp8 bl8; do
  if [ $tag = fp8 ]; then A="--steps 4 --warmup 3 --model roberta-large --task masked-lm --seq_len 512 --batch_size 64 --dtype fp8"; M=embed_fwd; else A="--model bert-large-uncased --seq_len 512 --batch_size 8 --steps 6 --warmup 3"; M=embed_fwd; fi
  rm -rf gpurun_out/tl_$tag
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl_$tag -o run -- python bench.py $A > gpurun_out/tl_$tag.log 2>&1 || { tail -20 gpurun_out/tl_$tag.log; exit 1; }
  f=$(find gpurun_out/tl_$tag -name "*kernel_trace.csv" | head -1)
  cp "$f" gpurun_out/trace_${tag}_r6c.csv
  rm -rf gpurun_out/tl_$tag
  python tools/timeline.py gpurun_out/trace_${tag}_r6c.csv --steps 3 --marker $M --top 30 > gpurun_out/timeline_${tag}_r6c.txt || exit 1
  head -75 gpurun_out/timeline_${tag}_r6c.txt
done
