#!/bin/bash
# regression check: headline bench at HEAD vs the round-4 final-evidence commit (worktree ab_old, built in-tree),
# interleaved x2 on one box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for r in 1 2; do
  timeout -k 10 200 python bench.py 2>/dev/null | tail -1 | cut -c1-110 | sed "s/^/HEAD /" || exit 1
  (cd ab_old && timeout -k 10 200 python bench.py 2>/dev/null | tail -1 | cut -c1-110 | sed "s/^/ad1768f /") || exit 1
done
