"""Time transpose_many over bert-base's 48 encoder weights (one Wᵀ refresh of the whole model) vs torch copies.
    python tools/bench_transpose.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from huggingface_sagemaker_tensorflow_distributed_amd.ops import hip  # noqa: E402

dev = "cuda"
shapes = [(2304, 768), (768, 768), (3072, 768), (768, 3072)] * 12
srcs = [torch.randn(r, c, device=dev).bfloat16() for r, c in shapes]
dsts = [torch.empty(c, r, device=dev, dtype=torch.bfloat16) for r, c in shapes]
desc, tiles = [], 0
for s, d in zip(srcs, dsts):
    desc.append([s.data_ptr(), d.data_ptr(), s.shape[0], s.shape[1], tiles])
    tiles += ((s.shape[0] + 63) // 64) * ((s.shape[1] + 63) // 64)
dt = torch.tensor(desc, dtype=torch.int64, device=dev)
nbytes = 2 * sum(s.numel() * 2 for s in srcs)


def timed(fn, it=20):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(it):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / it * 1e3


t_ours = timed(lambda: hip._C.transpose_many(dt, tiles))
t_torch = timed(lambda: [d.copy_(s.t()) for s, d in zip(srcs, dsts)])
assert all(torch.equal(d, s.t()) for s, d in zip(srcs, dsts))
print(f"transpose_many: {t_ours:.1f} us ({nbytes / t_ours / 1e6:.2f} TB/s); torch copies: {t_torch:.1f} us "
      f"({nbytes / t_torch / 1e6:.2f} TB/s); {nbytes / 1e6:.0f} MB moved")
