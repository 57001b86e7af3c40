# Two DP ranks sharing the one GPU of a gpurun box (gloo transport: RCCL refuses two ranks on one device):
# exercises the world>1 GPU training path (bucket hooks from the HIP backward, async all-reduce, max-over-ranks
# timing) end to end. Not a performance number.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp HSD_DIST_BACKEND=gloo
mkdir -p gpurun_out
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --batch_size 64 > gpurun_out/two_ranks.log 2>&1 || { tail -30 gpurun_out/two_ranks.log; exit 1; }
grep '"metric"' gpurun_out/two_ranks.log
