for c in "--model bert-large-uncased --seq_len 512 --batch_size 8" "--batch_size 64" "--batch_size 256"; do
  for mk in 4 8 16 4 8 16; do
    echo -n "min_kt=$mk $c: "
    HSD_WGRAD_MIN_KT=$mk timeout -k 10 200 python bench.py --steps 20 --warmup 5 $c 2>/dev/null | grep metric | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'
  done
done
