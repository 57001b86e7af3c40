"""LayerNorm forward A/B at the BERT-base B=1024 shape: one-row-per-wave kernel (HSD_LN_FWD_RPW=1) vs the
multi-row kernel at several rows-per-wave; outputs must be bit-identical. -> gpurun_out/bench_ln.json"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from huggingface_sagemaker_tensorflow_distributed_amd.ops import hip  # noqa: E402

C_ = hip._C
dev = "cuda"
T, H = 131072, 768


def timeit(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(iters):
        fn()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / iters * 1e3


y = torch.randn(T, H, device=dev).bfloat16()
r = torch.randn(T, H, device=dev).bfloat16()
g = (torch.rand(H, device=dev) + 0.5).bfloat16()
b = torch.randn(H, device=dev).bfloat16()
res = {}
outs = {}
for mode in ["1", "8", "16", "0"]:
    os.environ["HSD_LN_FWD_RPW"] = mode
    hip._C.refresh_env()  # launch knobs are cached (common.h HSD_KNOB)
    for p in (0.0, 0.1):
        for with_res in (False, True):
            z = torch.empty_like(y) if with_res else None
            o = torch.empty_like(y)
            mean = torch.empty(T, device=dev)
            rstd = torch.empty(T, device=dev)
            fn = lambda: C_.ln_fwd(y, r if with_res else None, g, b, z, o, mean, rstd, 1e-12, p, 7)  # noqa: E731
            fn()
            torch.cuda.synchronize()
            key = f"p{p}_res{int(with_res)}"
            outs.setdefault(key, []).append((mode, o.clone(), mean.clone(), rstd.clone()))
            ts = sorted(timeit(fn) for _ in range(3))
            us = ts[1]
            nbytes = T * H * 2 * (2 + (2 if with_res else 0))
            res[f"rpw{mode}_{key}_us"] = round(us, 1)
            res[f"rpw{mode}_{key}_TBs"] = round(nbytes / us / 1e6, 2)
for key, lst in outs.items():
    m0, o0, mu0, rs0 = lst[0]
    for mode, o, mu, rs in lst[1:]:
        res[f"same_{key}_rpw{mode}"] = bool(torch.equal(o, o0) and torch.equal(mu, mu0) and torch.equal(rs, rs0))
        if not res[f"same_{key}_rpw{mode}"]:
            bad = (o != o0).any(1).nonzero().flatten()
            res[f"diff_{key}_rpw{mode}"] = dict(
                o=(o.float() - o0.float()).abs().max().item(), mu=(mu - mu0).abs().max().item(),
                rs=(rs - rs0).abs().max().item(), nbad_rows=int(bad.numel()), first=bad[:4].tolist(),
                nan0=bool(o0.isnan().any()), nan=bool(o.isnan().any()))
print(json.dumps(res, indent=1))
os.makedirs("gpurun_out", exist_ok=True)
json.dump(res, open("gpurun_out/bench_ln.json", "w"), indent=1)
