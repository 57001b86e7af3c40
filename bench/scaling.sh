#!/bin/bash
# Headline scaling curve: whole-node seq/s for bert-base S=128 bf16 at N = 1, 2, 4, 8 MI355X (one rank per
# GPU over RCCL/xGMI). Each N runs bench.py exactly as the driver does; results -> bench/scaling_<N>.json.
#   bash bench/scaling.sh [steps] [warmup]
set -eo pipefail
cd "$(dirname "$0")/.."
STEPS=${1:-20}
WARM=${2:-5}
for N in 1 2 4 8; do
  if [ "$N" -eq 1 ]; then
    timeout -k 10 900 python bench.py --gpus 1 --steps "$STEPS" --warmup "$WARM" | tail -1 | tee bench/scaling_1.json
  else
    timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" --master-addr 127.0.0.1 \
      --master-port $((29600 + N)) bench.py --gpus "$N" --steps "$STEPS" --warmup "$WARM" | tail -1 | tee "bench/scaling_${N}.json"
  fi
done
python - <<'PY'
import json
rows = [json.load(open(f"bench/scaling_{n}.json")) for n in (1, 2, 4, 8)]
base = rows[0]["value"]
for r in rows:
    print(f'N={r["n_gpus"]}: {r["value"]:10.1f} seq/s  ({r["value"] / (base * r["n_gpus"]) * 100:5.1f}% weak-scaling eff.)')
PY
