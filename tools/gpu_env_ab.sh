#!/bin/bash
# Interleaved env-knob A/B of bench.py on one box: ENVS="A=0 A=1" CONFIGS="--batch_size 32|--model ..." (| separated)
# REPS=2 bash tools/gpu_env_ab.sh  -> gpurun_out/env_ab.log (seq/s, ms/step per run)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
out=gpurun_out/env_ab.log
: > $out
IFS='|' read -ra cfgs <<< "${CONFIGS:---steps 20 --warmup 5}"
for r in $(seq ${REPS:-2}); do
  for c in "${cfgs[@]}"; do
    for e in $ENVS; do
      v=$(env $e timeout -k 10 300 python bench.py $c 2>/dev/null | tail -1 | python -c "import json,sys; j=json.loads(sys.stdin.read()); print(j['value'], j['ms_per_step'])") || exit 1
      echo "$c [$e] : $v" | tee -a $out
    done
  done
done
