"""Epilogue cost on one NT GEMM shape (default the FFN1 forward, T x 3072 x 768; EPI_N / EPI_K / EPI_T override):
store / bias / bias+GELU (2 outputs) / bias+GELU+GELU' (2 outputs) / residual add (aux read) / dropout+residual at
p = 0 and 0.1 / GELU' product, interleaved rounds in one process.   python tools/epi_cost.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from huggingface_sagemaker_tensorflow_distributed_amd.ops import hip  # noqa: E402

C_ = hip._C
dev = "cuda"
T, N, K = (int(os.environ.get(k, d)) for k, d in (("EPI_T", "131072"), ("EPI_N", "3072"), ("EPI_K", "768")))
rnd = lambda *s: (torch.rand(*s, device=dev) * 2 - 1).bfloat16()  # noqa: E731
a, b, bias, aux = rnd(T, K), rnd(N, K) * 0.05, rnd(N), rnd(T, N)
c, c2 = torch.empty(T, N, device=dev, dtype=torch.bfloat16), torch.empty(T, N, device=dev, dtype=torch.bfloat16)
db = torch.zeros(N, device=dev)
cases = {
    "E0_store": lambda: C_.gemm2(a, b, c, 0, 0, 0, None, None, None, 0.0, 0, 1, None, None),
    "E1_bias": lambda: C_.gemm2(a, b, c, 0, 0, 1, bias, None, None, 0.0, 0, 1, None, None),
    "E2_bias_gelu_2out": lambda: C_.gemm2(a, b, c, 0, 0, 2, bias, None, c2, 0.0, 0, 1, None, None),
    "E8_bias_gelu_gelud_2out": lambda: C_.gemm2(a, b, c, 0, 0, 8, bias, None, c2, 0.0, 0, 1, None, None),
    "E4_res_auxread": lambda: C_.gemm2(a, b, c, 0, 0, 4, None, aux, None, 0.0, 0, 1, None, None),
    "E9_mul_auxread_dbias": lambda: C_.gemm2(a, b, c, 0, 0, 9, None, aux, None, 0.0, 0, 1, None, db),
    "E3_bias_res_p0": lambda: C_.gemm2(a, b, c, 0, 0, 3, bias, aux, None, 0.0, 7, 1, None, None),
    "E3_bias_drop_res_p01": lambda: C_.gemm2(a, b, c, 0, 0, 3, bias, aux, None, 0.1, 7, 1, None, None),
}


def timeit(fn, iters=8):
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    st.record()
    for _ in range(iters):
        fn()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / iters * 1e3


t = {k: [] for k in cases}
for _ in range(3):
    for k, fn in cases.items():
        t[k].append(timeit(fn))
res = {k: round(min(v), 1) for k, v in t.items()}
print(json.dumps(res))
