#!/bin/bash
# PMC passes (kernel-trace + pmc only, one counter set per run) over the headline layer's heaviest GEMMs at T = 131072:
# MFMA busy vs GPU active, L2 hit rate and HBM/fabric bytes, CU->L2 request counts.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/pmc4
for g in ${GEMMS:-ffn1_fwd_gelu_d ffn2_dgrad_mul_dbias ffn1_dgrad_res qkv_fwd_bias out_fwd_drop_res ffn1_wgrad}; do
  i=0
  for set in "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE" \
             "FETCH_SIZE TCC_HIT_sum" "WRITE_SIZE TCC_MISS_sum TCC_EA0_RDREQ_sum" "TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum"; do
    i=$((i+1))
    timeout -s KILL 60 rocprofv3 --kernel-trace --pmc $set --output-format csv -d gpurun_out/pmc4/${g}_$i -o run -- python tools/gemm_pmc_one.py $g > gpurun_out/pmc4_${g}_$i.log 2>&1 || { echo "pmc failed $g $i"; tail -5 gpurun_out/pmc4_${g}_$i.log; exit 1; }
  done
done
python - <<'PY'
import csv, glob, os, collections
out = ["gemm\tkernel\tcounter\tmean_per_dispatch\tmean_duration_ns"]
for d in sorted(glob.glob("gpurun_out/pmc4/*")):
    g = os.path.basename(d).rsplit("_", 1)[0]
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        agg = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            if "g2::" not in r["Kernel_Name"]: continue
            agg[(r["Kernel_Name"].split("(")[0][-40:], r["Counter_Name"])].append(float(r["Counter_Value"]))
        for (k, c), v in sorted(agg.items()):
            out.append(f"{g}\t{k}\t{c}\t{sum(v)/len(v):.5g}")
open("gpurun_out/pmc4_summary.tsv", "w").write("\n".join(out) + "\n")
print("\n".join(out))
PY
