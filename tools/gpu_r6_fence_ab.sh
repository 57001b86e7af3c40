# A/B: fork events without (default) / with (HSD_EVENT_SYSFENCE=1) the system-scope fence; bert-large B=8 and the
# headline, interleaved x2, then the timeline of the new default
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/fence_ab.log
for rep in 1 2; do
  for f in 1 0; do
    for cfg in "--model bert-large-uncased --seq_len 512 --batch_size 8 --steps 30 --warmup 5" "--steps 10 --warmup 3"; do
      HSD_EVENT_SYSFENCE=$f timeout -k 10 300 python bench.py $cfg > gpurun_out/fab.json 2>gpurun_out/fab.err || { tail -20 gpurun_out/fab.err; exit 1; }
      tail -1 gpurun_out/fab.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('sysfence=$f', '$cfg', d['value'], d['ms_per_step'])" | tee -a gpurun_out/fence_ab.log || exit 1
    done
  done
done
rm -rf gpurun_out/tl_bl8
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl_bl8 -o run -- python bench.py --model bert-large-uncased --seq_len 512 --batch_size 8 --steps 6 --warmup 3 > gpurun_out/tl_bl8.log 2>&1 || { tail -20 gpurun_out/tl_bl8.log; exit 1; }
f=$(find gpurun_out/tl_bl8 -name "*kernel_trace.csv" | head -1)
cp "$f" gpurun_out/trace_bl8_r6_nofence.csv
rm -rf gpurun_out/tl_bl8
python tools/timeline.py gpurun_out/trace_bl8_r6_nofence.csv --steps 4 --top 12
