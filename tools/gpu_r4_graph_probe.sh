#!/bin/bash
# Why is the captured step slower than eager at small batches? bench + kernel traces of both (bert-base B=32,
# bert-large S=512 B=8).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/gp
for cfg in "--batch_size 32" "--model bert-large-uncased --seq_len 512 --batch_size 8"; do
  for g in "" "--hip_graph"; do
    timeout -k 10 200 python bench.py --steps 30 --warmup 5 $cfg $g > gpurun_out/gp_bench.log 2>&1 || { tail -20 gpurun_out/gp_bench.log; exit 1; }
    echo "$cfg $g : $(tail -1 gpurun_out/gp_bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
i=0
for cfg in "--batch_size 32" "--batch_size 32 --hip_graph"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gp/t$i -o run -- python bench.py --steps 10 --warmup 3 $cfg > gpurun_out/gp_t$i.log 2>&1 || { tail -20 gpurun_out/gp_t$i.log; exit 1; }
done
python tools/trace_gaps.py gpurun_out/gp/t1 gpurun_out/gp/t2
