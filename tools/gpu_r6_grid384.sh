# HEAD with the 384-workgroup small-step weight-gradient target: GPU tier + smoke + bert-large B=8 / bert-base B=32 /
# headline benches (B=8 and B=32 also at the old 192 target, same box)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=r6grid NO_TESTS= bash tools/gpu_r6_suite.sh || exit 1
: > gpurun_out/grid384.log
for r in 1 2; do
  for g in default 192; do
    for cfg in "--model bert-large-uncased --seq_len 512 --batch_size 8 --steps 30 --warmup 5" "--batch_size 32 --steps 50 --warmup 10"; do
      if [ $g = default ]; then E="X=0"; else E="HSD_WGRAD_MIN_GRID=$g"; fi
      env $E timeout -k 10 300 python bench.py $cfg > gpurun_out/g.json 2>gpurun_out/g.err || { tail -20 gpurun_out/g.err; exit 1; }
      tail -1 gpurun_out/g.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('grid=$g $cfg', d['value'], d['ms_per_step'])" | tee -a gpurun_out/grid384.log || exit 1
    done
  done
done
