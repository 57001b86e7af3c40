"""A/B of gemm2 schedule variants (HSD_G2_SYNC) in ONE process, interleaved rounds (§5.4 rule 24)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from huggingface_sagemaker_tensorflow_distributed_amd.ops import hip  # noqa: E402

C_ = hip._C
T = int(os.environ.get("AB_T", "32768"))
variants = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "0,1").split(",")]
AB_VAR = os.environ.get("AB_VAR", "HSD_G2_SYNC")  # environment variable the variants set


def timeit(fn, iters=20):
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    st.record()
    for _ in range(iters):
        fn()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / iters * 1e-3


cases = {}
bufs = {}
for name, (N, K) in {"qkv": (2304, 768), "out": (768, 768), "ffn1": (3072, 768), "ffn2": (768, 3072)}.items():
    x = torch.randn(T, K, device="cuda").bfloat16()
    w = torch.randn(N, K, device="cuda").bfloat16()
    b = torch.randn(N, device="cuda").bfloat16()
    y = torch.empty(T, N, device="cuda", dtype=torch.bfloat16)
    y2 = torch.empty_like(y)
    dy = torch.randn(T, N, device="cuda").bfloat16()
    wt = w.t().contiguous()
    dx = torch.empty(T, K, device="cuda", dtype=torch.bfloat16)
    gw = torch.zeros(N, K, device="cuda")
    sp = C_.gemm2_splits(N, K, T)
    ws = torch.empty(sp * N * K, device="cuda")
    fl = 2 * T * N * K
    bufs[f"{name}_fwd"] = [y]
    bufs[f"{name}_gelu"] = [y, y2]
    bufs[f"{name}_dgrad"] = [dx]
    bufs[f"{name}_wgrad"] = [gw]
    if os.environ.get("AB_ONLY_WGRAD"):
        cases[f"{name}_wgrad"] = (fl, lambda dy=dy, x=x, gw=gw, sp=sp, ws=ws: C_.gemm2(dy, x, gw, 1, 1, 7, None, None, None, 0.0, 0, sp, ws, None))
        continue
    cases[f"{name}_fwd"] = (fl, lambda x=x, w=w, y=y: C_.gemm2(x, w, y, 0, 0, 0, None, None, None, 0.0, 0, 1, None, None))
    res_in = torch.randn(T, N, device="cuda").bfloat16()
    resK = torch.randn(T, K, device="cuda").bfloat16()
    bufs[f"{name}_droppres"] = [y]
    bufs[f"{name}_dgrad_res"] = [dx]
    bufs[f"{name}_dgrad_dgelu"] = [dx]
    cases[f"{name}_droppres"] = (fl, lambda x=x, w=w, y=y, b=b, r=res_in: C_.gemm2(x, w, y, 0, 0, 3, b, r, None, 0.1, 5, 1, None, None))
    cases[f"{name}_dgrad_res"] = (fl, lambda dy=dy, wt=wt, dx=dx, r=resK: C_.gemm2(dy, wt, dx, 0, 0, 4, None, r, None, 0.0, 0, 1, None, None))
    if K % 256 == 0:
        cases[f"{name}_dgrad_dgelu"] = (fl, lambda dy=dy, wt=wt, dx=dx, r=resK: C_.gemm2(dy, wt, dx, 0, 0, 5, None, r, None, 0.0, 0, 1, None, None))
    if name == "ffn1":
        cases[f"{name}_gelu"] = (fl, lambda x=x, w=w, y=y, b=b, y2=y2: C_.gemm2(x, w, y, 0, 0, 2, b, None, y2, 0.0, 0, 1, None, None))
    cases[f"{name}_dgrad"] = (fl, lambda dy=dy, wt=wt, dx=dx: C_.gemm2(dy, wt, dx, 0, 0, 0, None, None, None, 0.0, 0, 1, None, None))
    if os.environ.get("AB_NO_WGRAD"):
        continue
    cases[f"{name}_wgrad"] = (fl, lambda dy=dy, x=x, gw=gw, sp=sp, ws=ws: C_.gemm2(dy, x, gw, 1, 1, 7, None, None, None, 0.0, 0, sp, ws, None))
outs = {"fwd": lambda: y, "gelu": lambda: y2, "dgrad": lambda: dx, "wgrad": lambda: gw}
# correctness of every variant against variant 0 (same inputs): run each case, snapshot its output
bad = []
for k, (fl, fn) in cases.items():
    snaps = []
    for v in variants:
        os.environ[AB_VAR] = str(v)
        hip._C.refresh_env()  # launch knobs are cached (common.h HSD_KNOB)
        for t in list(bufs[k]):
            t.zero_()
        fn()
        torch.cuda.synchronize()
        snaps.append([t.float().clone() for t in bufs[k]])
    for vi, sn in enumerate(snaps[1:], 1):
        for a, b in zip(snaps[0], sn):
            d = (a - b).abs().max().item() / (a.abs().max().item() + 1e-6)
            if d > 1e-2:
                bad.append((k, variants[vi], d))
print("variant mismatches:", bad, flush=True)
res = {k: {v: [] for v in variants} for k in cases}
for rnd in range(3):
    for k, (fl, fn) in cases.items():
        for v in variants:
            os.environ[AB_VAR] = str(v)
            hip._C.refresh_env()  # launch knobs are cached (common.h HSD_KNOB)
            res[k][v].append(fl / timeit(fn) / 1e12)
for k in cases:
    print(k, "  ".join(f"v{v}: {max(res[k][v]):7.1f} (med {sorted(res[k][v])[1]:7.1f})" for v in variants), flush=True)
