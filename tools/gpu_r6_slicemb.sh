# Adam slice size after the fork-deferred slices (HSD_OPT_BUCKET_MB 8 / 16 / 32): bert-large B=8 and the headline
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
: > gpurun_out/slicemb_ab.log
for r in 1 2; do
  for mb in 16 8 32; do
    for cfg in "--model bert-large-uncased --seq_len 512 --batch_size 8 --steps 30 --warmup 5" "--steps 10 --warmup 3"; do
      HSD_OPT_BUCKET_MB=$mb timeout -k 10 300 python bench.py $cfg > gpurun_out/sm.json 2>gpurun_out/sm.err || { tail -20 gpurun_out/sm.err; exit 1; }
      tail -1 gpurun_out/sm.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('HSD_OPT_BUCKET_MB=$mb $cfg', d['value'], d['ms_per_step'])" | tee -a gpurun_out/slicemb_ab.log || exit 1
    done
  done
done
