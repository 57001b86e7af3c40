# bert-large B=8 knobs re-checked at HEAD: weight-gradient grid target (HSD_WGRAD_MIN_GRID), gemm2s stages / waves
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
: > gpurun_out/bl8sweep.log
A="--model bert-large-uncased --seq_len 512 --batch_size 8 --steps 30 --warmup 5"
for r in 1 2; do
  for e in "X=0" "HSD_WGRAD_MIN_GRID=128" "HSD_WGRAD_MIN_GRID=256" "HSD_WGRAD_MIN_GRID=384" "HSD_G2S_KW=1" "HSD_G2S_STAGES=4"; do
    env $e timeout -k 10 300 python bench.py $A > gpurun_out/sw.json 2>gpurun_out/sw.err || { tail -20 gpurun_out/sw.err; exit 1; }
    tail -1 gpurun_out/sw.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$e bert-large B=8', d['value'], d['ms_per_step'])" | tee -a gpurun_out/bl8sweep.log || exit 1
  done
done
