#!/bin/bash
# PMC of the fp8 GEMMs of the roberta-large MLM step: per shape, kernel trace + one counter set
# per rocprofv3 run (each within the per-block limits: <= 8 SQ, <= 4 TCC), summarised into gpurun_out/pmc_gemm8.tsv
# (MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs), VALU / MFMA instructions, bytes).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
SETS=("SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
      "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INST_CYCLES_VMEM SQ_INSTS_SALU GRBM_COUNT"
      "FETCH_SIZE"
      "WRITE_SIZE")
for w in ${SHAPES8:-qkv_fwd out_fwd ffn1_fwd ffn2_fwd ffn2_dgrad qkv_dgrad wgrad_ffn}; do
  for i in "${!SETS[@]}"; do
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc ${SETS[$i]} --output-format csv -d gpurun_out/pmc8_${w}_$i -o run \
      -- python tools/gemm8_pmc_one.py $w > gpurun_out/pmc8_${w}_$i.log 2>&1 || { echo "pmc failed $w $i"; tail -5 gpurun_out/pmc8_${w}_$i.log; exit 1; }
  done
done
python - <<'PY'
import csv, glob, os, collections
rows = collections.defaultdict(dict)
for d in sorted(glob.glob("gpurun_out/pmc8_*")):
    if not os.path.isdir(d):
        continue
    shape = os.path.basename(d)[len("pmc8_"):].rsplit("_", 1)[0]
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        agg = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            if "gemm8" not in r["Kernel_Name"]:
                continue
            agg[(r["Kernel_Name"].split("(")[0][-40:], r["Counter_Name"])].append(float(r["Counter_Value"]))
        for (k, c), v in agg.items():
            rows[(shape, k)][c] = sum(v) / len(v)
out = ["shape\tkernel\tmfma_busy_pct\tvalu_per_mfma\tlds_conflict_pct\tfetch_MB\twrite_MB\t" +
       "\t".join(["SQ_BUSY_CYCLES", "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_LDS",
                  "SQ_WAIT_INST_LDS", "SQ_WAVE_CYCLES", "GRBM_GUI_ACTIVE"])]
for (shape, k), c in sorted(rows.items()):
    busy = c.get("SQ_BUSY_CYCLES", 0)
    mb = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0)
    # the round-5 formula (profiles/pmc_gemm_r5c.tsv): SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs)
    gui = c.get("GRBM_GUI_ACTIVE", 0)
    pct = 100.0 * mb / (gui / 8 * 1024) if gui else float("nan")
    vpm = c.get("SQ_INSTS_VALU", 0) / max(1.0, c.get("SQ_INSTS_MFMA", 0))
    conf = 100.0 * c.get("SQ_LDS_BANK_CONFLICT", 0) / max(1.0, c.get("SQ_LDS_IDX_ACTIVE", 0))
    out.append(f"{shape}\t{k}\t{pct:.1f}\t{vpm:.2f}\t{conf:.2f}\t{c.get('FETCH_SIZE', 0) / 1024:.0f}\t"
               f"{c.get('WRITE_SIZE', 0) / 1024:.0f}\t" +
               "\t".join(f"{c.get(x, 0):.4g}" for x in ["SQ_BUSY_CYCLES", "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_INSTS_VALU",
                                                         "SQ_INSTS_MFMA", "SQ_INSTS_LDS", "SQ_WAIT_INST_LDS",
                                                         "SQ_WAVE_CYCLES", "GRBM_GUI_ACTIVE"]))
open("gpurun_out/pmc_gemm8.tsv", "w").write("\n".join(out) + "\n")
print("\n".join(out))
PY
