"""gemm2 (8-phase 256-row-tile MFMA GEMM): correctness vs fp32 torch + TF/s vs hipBLASLt on BERT shapes.

    python tools/bench_gemm2.py [T]     -> gpurun_out/bench_gemm2.json
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from huggingface_sagemaker_tensorflow_distributed_amd.ops import hip  # noqa: E402

C_ = hip._C
dev = "cuda"


def bench(fn, iters=30, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(iters):
        fn()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / iters * 1e-3


def relerr(a, b):
    return ((a.float() - b.float()).abs().max() / (b.float().abs().max() + 1e-6)).item()


T = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
torch.manual_seed(0)
res = {}
# ---- correctness on odd shapes first
for (M, N, K) in [(300, 768, 128), (512, 2304, 768), (1000, 192 * 5, 64 * 3)]:
    x = torch.randn(M, K, device=dev).bfloat16()
    w = torch.randn(N, K, device=dev).bfloat16()
    b = torch.randn(N, device=dev).bfloat16()
    y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    C_.gemm2(x, w, y, 0, 0, 1, b, None, None, 0.0, 0, 1, None, None)
    ref = x.float() @ w.float().t() + b.float()
    e = relerr(y, ref)
    print(f"NT bias M={M} N={N} K={K} err={e:.2e}", flush=True)
    assert e < 1e-2, e
    # TT: C[N][K] += x^T... use A = dy [M][N] (K-dim = M), B = x [M][K]
    dy = torch.randn(M, N, device=dev).bfloat16()
    if N % 256 == 0 and K % 256 == 0 and M % 64 == 0:
        for epi in (6, 7):
            gw = torch.randn(N, K, device=dev)
            g0 = gw.clone()
            sp = C_.gemm2_splits(N, K, M)
            ws = torch.empty(sp * N * K, device=dev)
            C_.gemm2(dy, x, gw, 1, 1, epi, None, None, None, 0.0, 0, 0, ws, None)
            ref = g0 + dy.float().t() @ x.float()
            e = relerr(gw, ref)
            print(f"TT epi{epi} M={N} N={K} K={M} splits={sp} err={e:.2e}", flush=True)
            assert e < 1e-3, e

for name, (N, K) in {"qkv": (2304, 768), "out": (768, 768), "ffn1": (3072, 768), "ffn2": (768, 3072)}.items():
    x = torch.randn(T, K, device=dev).bfloat16()
    w = torch.randn(N, K, device=dev).bfloat16()
    wt = w.t().contiguous()
    dy = torch.randn(T, N, device=dev).bfloat16()
    b = torch.randn(N, device=dev).bfloat16()
    fl = 2 * T * N * K
    y = torch.empty(T, N, device=dev, dtype=torch.bfloat16)
    y2 = torch.empty(T, N, device=dev, dtype=torch.bfloat16)
    res_in = torch.randn(T, N, device=dev).bfloat16()
    dx = torch.empty(T, K, device=dev, dtype=torch.bfloat16)
    gw = torch.zeros(N, K, device=dev)
    sp = C_.gemm2_splits(N, K, T)
    ws = torch.empty(sp * N * K, device=dev)
    r = {}
    # correctness at full size
    C_.gemm2(x, w, y, 0, 0, 1, b, None, None, 0.0, 0, 1, None, None)
    r["fwd_err"] = relerr(y, x.float() @ w.float().t() + b.float())
    C_.gemm2(dy, wt, dx, 0, 0, 0, None, None, None, 0.0, 0, 1, None, None)
    r["dgrad_err"] = relerr(dx, dy.float() @ w.float())
    gw.zero_()
    C_.gemm2(dy, x, gw, 1, 1, 7, None, None, None, 0.0, 0, 0, ws, None)
    r["wgrad_err"] = relerr(gw, dy.float().t() @ x.float())
    # speed
    r["fwd_torch"] = fl / bench(lambda: torch.addmm(b, x, w.t())) / 1e12
    r["fwd_bias"] = fl / bench(lambda: C_.gemm2(x, w, y, 0, 0, 1, b, None, None, 0.0, 0, 1, None, None)) / 1e12
    r["fwd_store"] = fl / bench(lambda: C_.gemm2(x, w, y, 0, 0, 0, None, None, None, 0.0, 0, 1, None, None)) / 1e12
    r["fwd_gelu"] = fl / bench(lambda: C_.gemm2(x, w, y, 0, 0, 2, b, None, y2, 0.0, 0, 1, None, None)) / 1e12
    r["fwd_droppres"] = fl / bench(lambda: C_.gemm2(x, w, y, 0, 0, 3, b, res_in, None, 0.1, 7, 1, None, None)) / 1e12
    r["fwd_old"] = fl / bench(lambda: C_.gemm(x, w, y, 0, 0, 1, b, None, None, 0.0, 0, 1)) / 1e12
    r["dgrad_torch"] = fl / bench(lambda: dy @ w) / 1e12
    r["dgrad_store"] = fl / bench(lambda: C_.gemm2(dy, wt, dx, 0, 0, 0, None, None, None, 0.0, 0, 1, None, None)) / 1e12
    pre = torch.randn(T, K, device=dev).bfloat16()
    db = torch.zeros(K, device=dev)
    if K % 256 == 0:
        C_.gemm2(dy, wt, dx, 0, 0, 5, None, pre, None, 0.0, 0, 1, None, db)
        import math
        ref = (dy.float() @ w.float())
        pf = pre.float()
        gp = 0.5 * (1 + torch.erf(pf / math.sqrt(2))) + pf * torch.exp(-0.5 * pf * pf) / math.sqrt(2 * math.pi)
        ref = (ref.bfloat16().float() * gp)
        r["dgelu_err"] = relerr(dx, ref)
        r["dbias_err"] = relerr(db, dx.float().sum(0))
        r["dgrad_dgelu_dbias"] = fl / bench(lambda: C_.gemm2(dy, wt, dx, 0, 0, 5, None, pre, None, 0.0, 0, 1, None, db)) / 1e12
    r["dgrad_dgelu"] = fl / bench(lambda: C_.gemm2(dy, wt, dx, 0, 0, 5, None, pre, None, 0.0, 0, 1, None, None)) / 1e12
    C_.gemm2(x, w, y, 0, 0, 2, b, None, y2, 0.0, 0, 1, None, None)
    yf = x.float() @ w.float().t() + b.float()
    r["gelu_err"] = relerr(y2, torch.nn.functional.gelu(y.float()))
    r["dgrad_old"] = fl / bench(lambda: C_.gemm(dy, w, dx, 0, 1, 0, None, None, None, 0.0, 0, 1)) / 1e12
    r["wgrad_torch"] = fl / bench(lambda: dy.t() @ x) / 1e12
    r["wgrad_slab"] = fl / bench(lambda: C_.gemm2(dy, x, gw, 1, 1, 7, None, None, None, 0.0, 0, 0, ws, None)) / 1e12
    r["wgrad_atomic"] = fl / bench(lambda: C_.gemm2(dy, x, gw, 1, 1, 6, None, None, None, 0.0, 0, 0, None, None)) / 1e12
    for s2 in (sp // 2, sp * 2):
        if s2 >= 1:
            ws2 = torch.empty(s2 * N * K, device=dev)
            r[f"wgrad_slab_s{s2}"] = fl / bench(lambda: C_.gemm2(dy, x, gw, 1, 1, 7, None, None, None, 0.0, 0, s2,
                                                                  ws2, None)) / 1e12
    r["wgrad_old"] = fl / bench(lambda: C_.gemm(dy, x, gw, 1, 1, 6, None, None, None, 0.0, 0, 8)) / 1e12
    r["splits"] = sp
    res[name] = {k: (round(v, 1) if isinstance(v, float) and v > 1 else v) for k, v in r.items()}
    print(name, res[name], flush=True)
os.makedirs("gpurun_out", exist_ok=True)
json.dump(res, open("gpurun_out/bench_gemm2.json", "w"), indent=1)
