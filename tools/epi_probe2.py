"""Epilogue-bound probe: T x 3072 x K NT GEMMs (K = 64: one K-tile, the epilogue dominates; K = 768: the FFN1 shape)
for E0 / E1 / E2 / E8 / E9, persistent grid capped at 256 / 128 / 64 workgroups (HSD_G2_GRID). If an epilogue is
bound by chip-wide HBM write bandwidth, halving the grid halves its per-round cost; if it is bound per CU, it does not.
    python tools/epi_probe2.py -> one JSON line per (K, epi)"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from huggingface_sagemaker_tensorflow_distributed_amd.ops import hip  # noqa: E402

C_ = hip._C
dev = "cuda"
T, N = 131072, 3072
rnd = lambda *s: (torch.rand(*s, device=dev) * 2 - 1).bfloat16()  # noqa: E731


def timeit(fn, iters=6):
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    st.record()
    for _ in range(iters):
        fn()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / iters * 1e3


bias, aux = rnd(N), rnd(T, N)
c, c2 = torch.empty(T, N, device=dev, dtype=torch.bfloat16), torch.empty(T, N, device=dev, dtype=torch.bfloat16)
db = torch.zeros(N, device=dev)
for K in (64, 768):
    a, b = rnd(T, K), rnd(N, K) * 0.05
    cases = {
        0: lambda: C_.gemm2(a, b, c, 0, 0, 0, None, None, None, 0.0, 0, 1, None, None),
        1: lambda: C_.gemm2(a, b, c, 0, 0, 1, bias, None, None, 0.0, 0, 1, None, None),
        2: lambda: C_.gemm2(a, b, c, 0, 0, 2, bias, None, c2, 0.0, 0, 1, None, None),
        8: lambda: C_.gemm2(a, b, c, 0, 0, 8, bias, None, c2, 0.0, 0, 1, None, None),
        9: lambda: C_.gemm2(a, b, c, 0, 0, 9, None, aux, None, 0.0, 0, 1, None, db),
    }
    for epi, fn in cases.items():
        r = {}
        for g in ("256", "128", "64"):
            os.environ["HSD_G2_GRID"] = g
            hip._C.refresh_env()  # launch knobs are cached (common.h HSD_KNOB)
            r[g] = round(min(timeit(fn) for _ in range(2)), 1)
        os.environ.pop("HSD_G2_GRID")
        hip._C.refresh_env()  # launch knobs are cached (common.h HSD_KNOB)
        print(json.dumps({"K": K, "epi": epi, "us_by_grid": r}), flush=True)
