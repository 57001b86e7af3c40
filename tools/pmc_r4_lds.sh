#!/bin/bash
# LDS bank-conflict cycles vs LDS-array cycles (SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE) and LDS instruction counts
# of the weight-gradient (TT: both operands through ds_read_b64_tr_b16) and the long-K NT GEMMs, one pass each
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/pmclds
for g in ${GEMMS:-ffn1_wgrad ffn1_dgrad_res ffn1_fwd_gelu_d}; do
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmclds/$g -o run -- python tools/gemm_pmc_one.py $g > gpurun_out/pmclds_$g.log 2>&1 || { echo "pmc failed $g"; tail -5 gpurun_out/pmclds_$g.log; exit 1; }
done
python - <<'PY'
import csv, glob, os, collections
for d in sorted(glob.glob("gpurun_out/pmclds/*")):
    g = os.path.basename(d)
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        agg = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            if "g2::" not in r["Kernel_Name"]: continue
            agg[(r["Kernel_Name"].split("(")[0][-34:], r["Counter_Name"])].append(float(r["Counter_Value"]))
        for (k, c), v in sorted(agg.items()):
            print(f"{g}\t{k}\t{c}\t{sum(v)/len(v):.5g}")
PY
