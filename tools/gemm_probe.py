"""gemm2 vs hipBLASLt on square shapes and the B=1024 BERT-base shapes (interleaved rounds, one process).

    PROBE_SYNC=1,4,5 python tools/gemm_probe.py [T]     -> gpurun_out/gemm_probe.json

Square 4096^3 / 8192^3 tell whether the main loop or the short-K tile overheads (prologue, epilogue)
bound the BERT shapes (K = 768 is 12 K-tiles per output tile). PROBE_SYNC lists the HSD_G2_SYNC schedules
to compare (NT forward and TT wgrad alike); every schedule is checked against an fp32 reference.
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from huggingface_sagemaker_tensorflow_distributed_amd.ops import hip  # noqa: E402

C_ = hip._C
dev = "cuda"
T = int(sys.argv[1]) if len(sys.argv) > 1 else 131072
VARS = [int(v) for v in os.environ.get("PROBE_SYNC", "1").split(",")]
SHAPES = {"sq4096": (4096, 4096, 4096), "sq8192": (8192, 8192, 8192),
          "qkv": (T, 2304, 768), "out": (T, 768, 768), "ffn1": (T, 3072, 768),
          "ffn2": (T, 768, 3072), "ffn1_dgrad": (T, 768, 3072)}
if os.environ.get("PROBE_ONLY"):
    SHAPES = {k: v for k, v in SHAPES.items() if k in os.environ["PROBE_ONLY"].split(",")}


def timeit(fn, iters=10):
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    st.record()
    for _ in range(iters):
        fn()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / iters * 1e-3


def with_sync(v, fn):
    os.environ["HSD_G2_SYNC"] = str(v)
    hip._C.refresh_env()  # launch knobs are cached (common.h HSD_KNOB)
    try:
        return fn()
    finally:
        os.environ.pop("HSD_G2_SYNC", None)
        hip._C.refresh_env()  # launch knobs are cached (common.h HSD_KNOB)


torch.manual_seed(0)
cases = {}
for name, (M, N, K) in SHAPES.items():
    x = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
    w = (torch.rand(N, K, device=dev) * 2 - 1).bfloat16()
    y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    fl = 2.0 * M * N * K
    ref = x[:512].float() @ w.float().t()
    ref_t = x[-256:].float() @ w.float().t()
    c = dict(fl=fl, torch=lambda x=x, w=w: torch.mm(x, w.t()),
             ours=lambda x=x, w=w, y=y: C_.gemm2(x, w, y, 0, 0, 0, None, None, None, 0.0, 0, 1, None, None))
    for v in VARS:
        y.zero_()
        with_sync(v, c["ours"])
        torch.cuda.synchronize()
        c[f"err_s{v}"] = ((y[:512].float() - ref).abs().max() / ref.abs().max()).item()
        c[f"tail_s{v}"] = ((y[-256:].float() - ref_t).abs().max() / ref_t.abs().max()).item()
    if K % 256 == 0 and N % 256 == 0 and M % 256 == 0:
        # TT wgrad of the same product: dW[N][K] += dY^T X with tokens = M
        dy = (torch.rand(M, N, device=dev) * 2 - 1).bfloat16()
        gw = torch.zeros(N, K, device=dev)
        sp = C_.gemm2_splits(N, K, M)
        ws = torch.empty(sp * N * K, device=dev)
        c["wgrad"] = lambda dy=dy, x=x, gw=gw, sp=sp, ws=ws: C_.gemm2(dy, x, gw, 1, 1, 7, None, None, None, 0.0, 0, sp,
                                                                      ws, None)
        c["wgrad_torch"] = lambda dy=dy, x=x: torch.mm(dy.t(), x)
        wref = dy.float().t() @ x.float()
        for v in VARS:
            gw.zero_()
            with_sync(v, c["wgrad"])
            torch.cuda.synchronize()
            c[f"werr_s{v}"] = ((gw - wref).abs().max() / wref.abs().max()).item()
        del wref
    cases[name] = c
    print("checked", name, {k: f"{v:.2e}" for k, v in c.items() if k.startswith(("err", "tail", "werr"))}, flush=True)
res = {k: {} for k in cases}
for rnd in range(3):
    for k, c in cases.items():
        for v in VARS:
            res[k].setdefault(f"ours_s{v}", []).append(c["fl"] / with_sync(v, lambda: timeit(c["ours"])) / 1e12)
            if "wgrad" in c:
                res[k].setdefault(f"wgrad_s{v}", []).append(c["fl"] / with_sync(v, lambda: timeit(c["wgrad"])) / 1e12)
        res[k].setdefault("torch", []).append(c["fl"] / timeit(c["torch"]) / 1e12)
        if "wgrad" in c:
            res[k].setdefault("wgrad_torch", []).append(c["fl"] / timeit(c["wgrad_torch"]) / 1e12)
out = {}
for k, c in cases.items():
    out[k] = {kk: round(sorted(v)[len(v) // 2], 1) for kk, v in res[k].items()}
    out[k].update({kk: float(f"{vv:.2e}") for kk, vv in c.items() if kk.startswith(("err", "tail", "werr"))})
    print(k, out[k], flush=True)
os.makedirs("gpurun_out", exist_ok=True)
json.dump(out, open("gpurun_out/gemm_probe.json", "w"), indent=1)
