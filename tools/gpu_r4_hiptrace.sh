#!/bin/bash
# HIP API trace of bert-large S=512 B=8 (long-blocking runtime calls on the host = where the host waits on the GPU)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/hiptrace
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --output-format csv -d gpurun_out/hiptrace -o run -- python bench.py --model bert-large-uncased --seq_len 512 --batch_size 8 --steps 8 --warmup 4 > gpurun_out/hiptrace.log 2>&1 || { tail -5 gpurun_out/hiptrace.log; exit 1; }
tail -1 gpurun_out/hiptrace.log | cut -c1-120
f=$(find gpurun_out/hiptrace -name "*hip_api_trace.csv" | head -1)
python - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
print(list(rows[0].keys()))
d = collections.defaultdict(list)
for r in rows:
    d[r["Function"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
tot = sorted(((sum(v), k, len(v), max(v)) for k, v in d.items()), reverse=True)
for s, k, n, mx in tot[:25]:
    print(f"{s/1e6:9.2f} ms {n:7d} calls max {mx/1e3:9.1f} us  {k}")
PY
