"""fp32 bias-gradient column sums (colsum32) vs HSD_COLSUM_MIN_ROWS at the bert-large B = 8 shapes.
    python tools/colsum32_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from huggingface_sagemaker_tensorflow_distributed_amd.ops import hip  # noqa: E402

C_ = hip._C
for M, N in ((4096, 1024), (4096, 3072), (4096, 4096)):
    x = torch.randn(M, N, device="cuda")
    d = torch.zeros(N, device="cuda")
    for rows in (32, 64, 128, 256, 512):
        os.environ["HSD_COLSUM_MIN_ROWS"] = str(rows)
        C_.refresh_env()
        for _ in range(3):
            C_.colsum32(x, d)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(50):
            C_.colsum32(x, d)
        b.record()
        torch.cuda.synchronize()
        us = a.elapsed_time(b) / 50 * 1e3
        print(f"M={M} N={N} min_rows={rows}: {us:.1f} us ({M * N * 4 / us / 1e6:.2f} TB/s)", flush=True)
