#!/bin/bash
# PMC passes over the attention kernels (tools/attn_one.py; ATTN_SHAPE=B,S,heads selects the shape): kernel-trace + pmc only, one counter set per run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python tools/attn_one.py 0.1 5 > gpurun_out/attn_one.log 2>&1 || { cat gpurun_out/attn_one.log; exit 1; }
cat gpurun_out/attn_one.log
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $set --output-format csv -d gpurun_out/pmca_$i -o run -- python tools/attn_one.py 0.1 2 > gpurun_out/pmca_$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 gpurun_out/pmca_$i.log; exit 1; }
done
python - <<'PY'
import csv, glob, collections
out = []
for f in sorted(glob.glob("gpurun_out/pmca_*/**/*counter_collection.csv", recursive=True)):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        agg[(r["Kernel_Name"][:40], r["Counter_Name"])].append(float(r["Counter_Value"]))
    for (k, c), v in sorted(agg.items()):
        out.append(f"{k}\t{c}\t{sum(v)/len(v):.4g}")
open("gpurun_out/pmc_attn.tsv", "w").write("\n".join(out) + "\n")
print("\n".join(out))
PY
