"""Same operands, same NT shape, epilogue E0 (store) vs E1 (bias) vs E4 (residual): isolates the bias epilogue's cost.
    python tools/epi_bias_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from huggingface_sagemaker_tensorflow_distributed_amd.ops import hip  # noqa: E402

C_ = hip._C
dev = "cuda"


def timed(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3


for T, N, K in ((32768, 4096, 1024), (131072, 3072, 768), (131072, 2304, 768), (131072, 768, 3072)):
    x = torch.randn(T, K, device=dev).bfloat16()
    w = (torch.randn(N, K, device=dev) * 0.05).bfloat16()
    bias = torch.randn(N, device=dev).bfloat16()
    aux = torch.randn(T, N, device=dev).bfloat16()
    c = torch.empty(T, N, device=dev, dtype=torch.bfloat16)
    fns = {
        "E0": lambda: C_.gemm2(x, w, c, 0, 0, 0, None, None, None, 0.0, 0, 0, None, None),
        "E1": lambda: C_.gemm2(x, w, c, 0, 0, 1, bias, None, None, 0.0, 0, 0, None, None),
        "E4": lambda: C_.gemm2(x, w, c, 0, 0, 4, None, aux, None, 0.0, 0, 0, None, None),
        "gemm_fwd": lambda: hip.gemm_fwd(x, w, hip.EPI_BIAS, bias=bias),
    }
    res = {k: [] for k in fns}
    for _ in range(3):
        for k, f in fns.items():
            res[k].append(timed(f))
    fl = 2.0 * T * N * K
    print(f"T={T} N={N} K={K}: " + "  ".join(f"{k} {min(v):.1f} us ({fl / min(v) / 1e6:.0f} TF)" for k, v in res.items()),
          flush=True)
