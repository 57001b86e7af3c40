"""Embedding backward A/B at the BERT-base B=1024 S=128 shape: scalar kernel (HSD_EMBED_BWD_SCALAR=1) vs the
16-B kernel; gradients must agree to fp32 atomic-order noise. -> gpurun_out/bench_embed.json"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from huggingface_sagemaker_tensorflow_distributed_amd.ops import hip  # noqa: E402

C_ = hip._C
dev = "cuda"
B, S, H, V = 1024, 128, 768, 30522


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(iters):
        fn()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / iters * 1e3


torch.manual_seed(0)
ids = torch.randint(0, V, (B, S), device=dev)
pos = torch.arange(S, device=dev).unsqueeze(0).expand(B, S).contiguous()
tt = torch.zeros(B, S, dtype=torch.long, device=dev)
word = (torch.randn(V, H, device=dev) * 0.02).bfloat16()
pw = (torch.randn(512, H, device=dev) * 0.02).bfloat16()
tw = (torch.randn(2, H, device=dev) * 0.02).bfloat16()
g = (1 + 0.1 * torch.randn(H, device=dev)).bfloat16()
be = (0.1 * torch.randn(H, device=dev)).bfloat16()
out = torch.empty(B * S, H, device=dev, dtype=torch.bfloat16)
mean = torch.empty(B * S, device=dev)
rstd = torch.empty(B * S, device=dev)
C_.embed_fwd(ids, pos, tt, word, pw, tw, g, be, out, mean, rstd, 1e-12, 0.1, 5)
dout = torch.randn(B * S, H, device=dev).bfloat16()
res = {}
grads = {}
for mode in ("scalar", "vec16"):
    if mode == "scalar":
        os.environ["HSD_EMBED_BWD_SCALAR"] = "1"
        hip._C.refresh_env()  # launch knobs are cached (common.h HSD_KNOB)
    else:
        os.environ.pop("HSD_EMBED_BWD_SCALAR", None)
        hip._C.refresh_env()  # launch knobs are cached (common.h HSD_KNOB)
    gw, gp, gt = torch.zeros(V, H, device=dev), torch.zeros(512, H, device=dev), torch.zeros(2, H, device=dev)
    gg, gb = torch.zeros(H, device=dev), torch.zeros(H, device=dev)
    fn = lambda: C_.embed_bwd(dout, ids, pos, tt, word, pw, tw, g, mean, rstd, gw, gp, gt, gg, gb, B, S, True, 0.1, 5)  # noqa: E731
    for _ in (gw, gp, gt, gg, gb):
        pass
    fn()
    torch.cuda.synchronize()
    grads[mode] = [t.clone() for t in (gw, gp, gt, gg, gb)]
    res[f"{mode}_us"] = round(sorted(timeit(fn) for _ in range(3))[1], 1)
for name, a, b in zip(("word", "pos", "type", "gamma", "beta"), grads["scalar"], grads["vec16"]):
    res[f"rel_{name}"] = float((a - b).abs().max() / a.abs().max().clamp(min=1e-30))
print(json.dumps(res, indent=1))
os.makedirs("gpurun_out", exist_ok=True)
json.dump(res, open("gpurun_out/bench_embed.json", "w"), indent=1)
