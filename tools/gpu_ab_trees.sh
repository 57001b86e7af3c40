#!/bin/bash
# Same-box A/B of this tree against a reference checkout in ab_base/ (git worktree of an earlier commit, built in place):
# interleaved runs of each configuration, base first. Usage: bash tools/gpu_ab_trees.sh <rounds> <name>:<bench args>...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rounds=$1; shift
out=gpurun_out/ab_trees.log
: > $out
for r in $(seq $rounds); do
  for spec in "$@"; do
    name=${spec%%:*}; args=${spec#*:}
    for tree in ab_base .; do
      v=$(cd $tree && timeout -k 10 400 python bench.py $args 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])") || { echo "bench failed: $tree $name"; exit 1; }
      echo "$name tree=$tree round=$r seq_s,ms=$v" | tee -a $out
    done
  done
done
