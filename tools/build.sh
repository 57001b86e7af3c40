#!/bin/bash
# Build _C.so and _C_debug.so in-tree; print the first compiler errors on failure.
cd "$(dirname "$0")/.."
for dbg in False True; do
  out=$(python -c "from huggingface_sagemaker_tensorflow_distributed_amd import _build; print(_build.build(debug=$dbg))" 2>&1)
  if [ $? -ne 0 ]; then echo "$out" | grep -E "error" | head -15; exit 1; fi
done
echo "build ok"
