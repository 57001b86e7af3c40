#!/bin/bash
# Round-3 evidence refresh: GEMMs vs hipBLASLt at HEAD, bert-large S=512 at B = 64 / 128, bert-base B = 256 / 512.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python tools/vs_hipblaslt.py > gpurun_out/vs_hipblaslt.log 2>&1 || { tail -5 gpurun_out/vs_hipblaslt.log; exit 1; }
for b in "--model bert-large-uncased --seq_len 512 --batch_size 64" "--model bert-large-uncased --seq_len 512 --batch_size 128" "--batch_size 256" "--batch_size 512"; do
  echo -n "$b: "
  timeout -k 10 300 python bench.py $b --steps 15 --warmup 4 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d[\"value\"], d[\"ms_per_step\"])" || exit 1
done
