"""Microbenchmark: hand-written MFMA GEMM vs torch/hipBLASLt on the BERT-base training shapes."""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from huggingface_sagemaker_tensorflow_distributed_amd.ops import hip  # noqa: E402

C_ = hip._C
dev = "cuda"


def bench(fn, iters=20, warm=5):
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


T = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
res = {}
for name, (N, K) in {"qkv": (2304, 768), "out": (768, 768), "ffn1": (3072, 768), "ffn2": (768, 3072)}.items():
    x = torch.randn(T, K, device=dev).bfloat16()
    w = torch.randn(N, K, device=dev).bfloat16()
    dy = torch.randn(T, N, device=dev).bfloat16()
    b = torch.randn(N, device=dev).bfloat16()
    fl = 2 * T * N * K
    y = torch.empty(T, N, device=dev, dtype=torch.bfloat16)
    dx = torch.empty(T, K, device=dev, dtype=torch.bfloat16)
    gw = torch.zeros(N, K, device=dev)
    r = {}
    r["fwd_torch"] = fl / bench(lambda: torch.addmm(b, x, w.t())) / 1e12
    r["fwd_hsd"] = fl / bench(lambda: C_.gemm(x, w, y, 0, 0, 1, b, None, None, 0.0, 0, 1)) / 1e12
    r["dgrad_torch"] = fl / bench(lambda: dy @ w) / 1e12
    r["dgrad_hsd"] = fl / bench(lambda: C_.gemm(dy, w, dx, 0, 1, 0, None, None, None, 0.0, 0, 1)) / 1e12
    r["wgrad_torch"] = fl / bench(lambda: dy.t() @ x) / 1e12
    for sp in (2, 4, 8):
        r[f"wgrad_big_s{sp}"] = fl / bench(lambda: C_.gemm_wgrad_variant(dy, x, gw, sp)) / 1e12
    tiles = ((N + 127) // 128) * ((K + 127) // 128)
    for sp in (1, 2, 4, 8, 16):
        if tiles * sp > 4096:
            break
        r[f"wgrad_hsd_s{sp}"] = fl / bench(lambda: C_.gemm(dy, x, gw, 1, 1, 6, None, None, None, 0.0, 0, sp)) / 1e12
    for v in range(8):
        r[f"fwd_v{v}"] = fl / bench(lambda: C_.gemm_variant(x, w, y, 0, 0, v)) / 1e12
        r[f"dgrad_v{v}"] = fl / bench(lambda: C_.gemm_variant(dy, w, dx, 0, 1, v)) / 1e12
    import os
    os.environ["HSD_GEMM_V1"] = "1"
    r["fwd_hsd_v1"] = fl / bench(lambda: C_.gemm(x, w, y, 0, 0, 1, b, None, None, 0.0, 0, 1)) / 1e12
    r["dgrad_hsd_v1"] = fl / bench(lambda: C_.gemm(dy, w, dx, 0, 1, 0, None, None, None, 0.0, 0, 1)) / 1e12
    del os.environ["HSD_GEMM_V1"]
    res[name] = {k: round(v, 1) for k, v in r.items()}
    print(name, res[name], flush=True)
json.dump(res, open("gpurun_out/bench_gemm.json", "w"), indent=1)
