#!/bin/bash
# Same-box A/B of the headline layer's GEMMs between ab_base/ (a worktree of an earlier commit, built in place) and this
# tree: tools/env_ab_gemm.py / env_ab_wgrad.py with a no-op switch, run from each tree's root, interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/tree_gemm_ab.log
: > $out
for r in 1 2; do
  for tree in ab_base .; do
    (cd $tree && timeout -k 10 300 python tools/env_ab_gemm.py HSD_TREE_AB_NOOP 0 2>/dev/null && timeout -k 10 300 python tools/env_ab_wgrad.py HSD_TREE_AB_NOOP 0 2>/dev/null) | sed "s/^/tree=$tree round=$r /" | tee -a $out || exit 1
  done
done
