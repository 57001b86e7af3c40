#!/bin/bash
# PMC passes over the S=128 attention forward/backward at the headline shape (B=1024, 12 heads), kernel-trace + pmc only.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/pmca4
i=0
for set in "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_WAVES" \
           "FETCH_SIZE TCC_HIT_sum" "WRITE_SIZE TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc $set --output-format csv -d gpurun_out/pmca4/p$i -o run -- python tools/attn_one.py 0.1 3 > gpurun_out/pmca4_$i.log 2>&1 || { echo "pmc failed $i"; tail -5 gpurun_out/pmca4_$i.log; exit 1; }
done
python - <<'PY'
import csv, glob, os, collections
out = ["pass\tkernel\tcounter\tmean_per_dispatch"]
for d in sorted(glob.glob("gpurun_out/pmca4/*")):
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        agg = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            if "a128" not in r["Kernel_Name"]: continue
            agg[(r["Kernel_Name"].split("(")[0][-36:], r["Counter_Name"])].append(float(r["Counter_Value"]))
        for (k, c), v in sorted(agg.items()):
            out.append(f"{os.path.basename(d)}\t{k}\t{c}\t{sum(v)/len(v):.5g}")
open("gpurun_out/pmca4_summary.tsv", "w").write("\n".join(out) + "\n")
print("\n".join(out))
PY
