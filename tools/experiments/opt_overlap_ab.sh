#!/bin/bash
# Optimizer overlapped with backward (HSD_OPT_OVERLAP=1, default) vs one Adam pass after backward (=0) on the
# headline config, the reference's own per-rank config and a mid batch.   bash tools/opt_overlap_ab.sh
set -e
run() {
  timeout -k 10 180 python bench.py --steps 20 --warmup 5 "$@" | grep '"metric"' | python -c \
    'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(json.dumps({"model": c["model"], "B": c["global_batch"], "S": c["seq_len"], "seq_s": d["value"], "ms": d["ms_per_step"]}))'
}
for cfg in "--batch_size 1024" "--model bert-large-uncased --seq_len 512 --batch_size 8" "--batch_size 64" \
           "--model bert-large-uncased --seq_len 512 --batch_size 64"; do
  for ov in 0 1 0 1; do
    echo -n "overlap=$ov "
    HSD_OPT_OVERLAP=$ov run $cfg
  done
done
