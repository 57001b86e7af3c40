#!/bin/bash
# A/B of env settings over bench.py configs: one line per (env, config). bash tools/ab_env_bench.sh "A=1 B=2" "A=0" ...
CONFIGS=${CONFIGS:-"--model bert-large-uncased --seq_len 512 --batch_size 8|--batch_size 64"}
IFS='|' read -ra CS <<< "$CONFIGS"
for envs in "$@"; do
  for c in "${CS[@]}"; do
    echo -n "[$envs] $c: "
    env $envs timeout -k 10 200 python bench.py --steps 20 --warmup 5 $c 2>/dev/null | grep metric | \
      python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])' || exit 1
  done
done
