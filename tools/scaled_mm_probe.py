"""Does hipBLASLt fp8 (torch._scaled_mm, OCP e4m3 / e5m2) run on this gfx950 box, and how fast, on the roberta-large
weight-gradient shapes (dW[N, K] = dyᵀ x over T = 32768 tokens)? Compares with our bf16 TT wgrad (gemm2)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from huggingface_sagemaker_tensorflow_distributed_amd.ops import hip  # noqa: E402

dev = "cuda"
T = 32768


def timeit(fn, iters=10):
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    st.record()
    for _ in range(iters):
        fn()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / iters * 1e3


for N, K in ((3072, 1024), (1024, 1024), (4096, 1024), (1024, 4096)):
    dy = torch.randn(T, N, device=dev).bfloat16()
    x = torch.randn(T, K, device=dev).bfloat16()
    out = {"N": N, "K": K}
    g = torch.zeros(N, K, device=dev)

    class G:
        buf = g
        mg = g
        p = None

    sp = hip._C.gemm2_splits(N, K, T)
    ws = torch.empty(sp * N * K, device=dev)
    out["ours_bf16_us"] = round(timeit(lambda: hip._C.gemm2(dy, x, g, 1, 1, 7, None, None, None, 0.0, 0, sp, ws, None)), 1)
    try:
        a = dy.t().contiguous().to(torch.float8_e5m2)          # [N, T] row-major
        b = x.t().contiguous().to(torch.float8_e4m3fn).t()     # [T, K] column-major
        one = torch.ones((), device=dev)
        r = torch._scaled_mm(a, b, scale_a=one, scale_b=one, out_dtype=torch.float32)
        ref = dy.float().t() @ x.float()
        out["scaled_mm_rel_err"] = round(float((r - ref).norm() / ref.norm()), 4)
        out["scaled_mm_us"] = round(timeit(lambda: torch._scaled_mm(a, b, scale_a=one, scale_b=one,
                                                                     out_dtype=torch.float32)), 1)
        a4 = dy.t().contiguous().to(torch.float8_e4m3fn)
        out["scaled_mm_e4m3_us"] = round(timeit(lambda: torch._scaled_mm(a4, b, scale_a=one, scale_b=one,
                                                                          out_dtype=torch.float32)), 1)
    except Exception as e:  # noqa: BLE001
        out["scaled_mm_error"] = repr(e)[:300]
    fl = 2.0 * T * N * K
    for k in ("ours_bf16_us", "scaled_mm_us", "scaled_mm_e4m3_us"):
        if k in out:
            out[k.replace("_us", "_TF")] = round(fl / out[k] / 1e6, 1)
    print(json.dumps(out), flush=True)
