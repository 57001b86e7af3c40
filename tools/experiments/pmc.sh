#!/bin/bash
# Counter collection for the GEMM kernels (kernel-trace + pmc only; never combined with sys/runtime traces).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
python -m huggingface_sagemaker_tensorflow_distributed_amd._build > gpurun_out/build.log 2>&1 || exit 1
rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
for w in fwd torch wgrad; do
  for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
             "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS" \
             "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum"; do
    tag=$(echo $set | cut -d' ' -f1)
    timeout -k 10 120 rocprofv3 --kernel-trace --pmc $set --output-format csv -d gpurun_out/pmc_${w}_${tag} -o run -- python tools/gemm_one.py $w > gpurun_out/pmc_${w}_${tag}.log 2>&1 || echo "pmc failed $w $tag"
  done
done
python - <<'PY'
import csv, glob, os, collections
out = []
for d in sorted(glob.glob("gpurun_out/pmc_*")):
    if not os.path.isdir(d): continue
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        agg = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            agg[(r["Kernel_Name"][:60], r["Counter_Name"])].append(float(r["Counter_Value"]))
        for (k, c), v in sorted(agg.items()):
            out.append(f"{d}\t{k}\t{c}\t{sum(v)/len(v):.4g}")
open("gpurun_out/pmc_summary.tsv", "w").write("\n".join(out) + "\n")
print("\n".join(out))
PY
