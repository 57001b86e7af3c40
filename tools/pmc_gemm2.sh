#!/bin/bash
# PMC passes over gemm2 NT (fwd, ffn1 shape) and TT (wgrad) — kernel-trace + pmc only, one pass per counter set.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp G1_T=${G1_T:-131072}
mkdir -p gpurun_out
for w in fwd wgrad; do
  i=0
  for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
             "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INST_CYCLES_VMEM TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $set --output-format csv -d gpurun_out/pmc2_${w}_$i -o run -- python tools/gemm2_one.py $w > gpurun_out/pmc2_${w}_$i.log 2>&1 || { echo "pmc failed $w $i"; tail -5 gpurun_out/pmc2_${w}_$i.log; exit 1; }
  done
done
python - <<'PY'
import csv, glob, os, collections
out = []
for d in sorted(glob.glob("gpurun_out/pmc2_*")):
    if not os.path.isdir(d): continue
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        agg = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            if "gemm2" not in r["Kernel_Name"]: continue
            agg[(r["Kernel_Name"][:48], r["Counter_Name"])].append(float(r["Counter_Value"]))
        for (k, c), v in sorted(agg.items()):
            out.append(f"{d}\t{k}\t{c}\t{sum(v)/len(v):.4g}")
open("gpurun_out/pmc2_summary.tsv", "w").write("\n".join(out) + "\n")
print("\n".join(out))
PY
