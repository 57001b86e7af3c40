#!/bin/bash
# two data-parallel ranks sharing the one GPU (gloo transport): the DP gradient path (bucket readiness from the weight-
# gradient side stream, all-reduce, Adam) at the headline per-rank batch; validation.ranks_in_sync must be true
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
HSD_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 3 --warmup 2 > gpurun_out/dp2_gloo.log 2>&1 || { tail -20 gpurun_out/dp2_gloo.log; exit 1; }
grep '"metric"' gpurun_out/dp2_gloo.log | python -c "import json,sys; d=json.loads(sys.stdin.readline()); print(d['value'], d['n_gpus'], d['config'], d.get('validation'))"
