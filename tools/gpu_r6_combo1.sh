# timelines (fp8 MLM, bert-large B=8) + the atomic weight-gradient A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_r6_atomic.sh || exit 1
bash tools/gpu_r6_tl2.sh || exit 1
