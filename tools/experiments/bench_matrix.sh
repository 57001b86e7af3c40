#!/bin/bash
# bench.py over a few configs (value, ms/step per line); extra env passes through.   bash tools/bench_matrix.sh
for c in "--model bert-large-uncased --seq_len 512 --batch_size 8" "--batch_size 64" "--batch_size 1024"; do
  for i in 1 2; do
    echo -n "$c: "
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 $c 2>/dev/null | grep metric | \
      python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'
  done
done
