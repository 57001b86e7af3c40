#!/bin/bash
# Kernel stats of one bench configuration: PROF_NAME=<tag> bash tools/prof_r4.sh <bench.py args...>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
n=${PROF_NAME:-prof}
rm -rf gpurun_out/$n
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$n -o run -- python bench.py "$@" > gpurun_out/$n.log 2>&1 || { tail -20 gpurun_out/$n.log; exit 1; }
tail -1 gpurun_out/$n.log | cut -c1-200
f=$(find gpurun_out/$n -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/kernel_stats_$n.csv
python - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:22]:
    print(f"{float(r['Percentage']):6.2f} {int(r['Calls']):6d} {float(r['AverageNs'])/1e3:9.1f}us  {r['Name'][:100]}")
PY
