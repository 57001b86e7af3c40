# bert-large B=8 at HEAD: stored-Wᵀ dgrads (HSD_WT=1), NT split-K off (HSD_G2_SPLITK=0), 256-tile NT (HSD_G2_SMALL=0)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
: > gpurun_out/bl8sweep3.log
A="--model bert-large-uncased --seq_len 512 --batch_size 8 --steps 30 --warmup 5"
for r in 1 2; do
  for e in "X=0" "HSD_WT=1" "HSD_G2_SPLITK=0" "HSD_G2_SMALL=0"; do
    env $e timeout -k 10 300 python bench.py $A > gpurun_out/sw.json 2>gpurun_out/sw.err || { tail -20 gpurun_out/sw.err; exit 1; }
    tail -1 gpurun_out/sw.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$e bert-large B=8', d['value'], d['ms_per_step'])" | tee -a gpurun_out/bl8sweep3.log || exit 1
  done
done
