#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/host_sync_probe.py --model bert-large-uncased --seq_len 512 --batch_size 8 > gpurun_out/hostprobe_bl8.log 2>&1 &&
timeout -k 10 200 python -u tools/host_sync_probe.py --model bert-base-uncased --seq_len 128 --batch_size 32 > gpurun_out/hostprobe_bb32.log 2>&1
grep -E "host enqueue|distinct" gpurun_out/hostprobe_*.log
