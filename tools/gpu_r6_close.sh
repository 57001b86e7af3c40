# Round-6 close-out at HEAD: smoke + GPU tier + headline bench, then our GEMMs vs hipBLASLt at the headline and
# bert-large B=8 shapes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=r6close bash tools/gpu_r6_suite.sh || exit 1
timeout -k 10 300 python tools/vs_hipblaslt.py 131072 768 > gpurun_out/vs_hipblaslt_r6_head.log 2>&1 || { tail -20 gpurun_out/vs_hipblaslt_r6_head.log; exit 1; }
tail -8 gpurun_out/vs_hipblaslt_r6_head.log | cut -c1-300
timeout -k 10 300 python tools/vs_hipblaslt.py 4096 1024 > gpurun_out/vs_hipblaslt_r6_bl8.log 2>&1 || { tail -20 gpurun_out/vs_hipblaslt_r6_bl8.log; exit 1; }
tail -8 gpurun_out/vs_hipblaslt_r6_bl8.log | cut -c1-300
