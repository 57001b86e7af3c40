#!/bin/bash
# Persistent NT GEMM start stagger (HSD_G2_STAGGER, 10 ns ticks): per-GEMM sweep (bit-identity checked), seam probe,
# headline bench A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
VALS=${VALS:-0,500,1000,1500,2000,3000}
timeout -k 10 400 python tools/env_ab_gemm.py HSD_G2_STAGGER $VALS > gpurun_out/stagger_ab.log 2>&1 || { tail -20 gpurun_out/stagger_ab.log; exit 1; }
cat gpurun_out/stagger_ab.log
for s in ${SEAM:-0 1500}; do
  HSD_G2_STAGGER=$s timeout -k 10 200 python tools/seam_probe.py > gpurun_out/seam_$s.log 2>&1 || { tail -20 gpurun_out/seam_$s.log; exit 1; }
  echo "stagger=$s"; grep -v '^#' gpurun_out/seam_$s.log | cut -c1-200
done
CONFIGS="--batch_size 1024" bash tools/ab_env_bench.sh ${BENCH:-"HSD_G2_STAGGER=0" "HSD_G2_STAGGER=1500" "HSD_G2_STAGGER=0" "HSD_G2_STAGGER=1500"}
