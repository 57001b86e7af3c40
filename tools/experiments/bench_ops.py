"""Microbenchmarks of the memory-bound + attention kernels at the BERT-base bench shape (B=256,S=128)."""
import json
import sys

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
    return st.elapsed_time(en) / iters * 1e3  # us


B, S, heads, H, I = 256, 128, 12, 768, 3072
T = B * S
res = {}
qkv = torch.randn(T, 3 * H, device=dev).bfloat16()
out = torch.empty(T, H, device=dev, dtype=torch.bfloat16)
lse = torch.empty(B * heads * S, device=dev)
dqkv = torch.empty_like(qkv)
dout = torch.randn(T, H, device=dev).bfloat16()
mask = torch.zeros(B, S, device=dev)
for p in (0.0, 0.1):
    res[f"attn_fwd_p{p}_us"] = bench(lambda: C_.attn_fwd(qkv, mask, out, lse, B, S, heads, p, 123))
    res[f"attn_bwd_p{p}_us"] = bench(lambda: C_.attn_bwd(qkv, mask, out, dout, lse, dqkv, None, B, S, heads, p, 123))
q, k, v = [t.view(B, S, heads, 64).transpose(1, 2).contiguous() for t in qkv.split(H, dim=1)]
q.requires_grad_(); k.requires_grad_(); v.requires_grad_()
sd = lambda: torch.nn.functional.scaled_dot_product_attention(q, k, v, dropout_p=0.0)  # noqa: E731
res["torch_sdpa_fwd_us"] = bench(sd)
o = sd()
g = torch.randn_like(o)
res["torch_sdpa_fwd_bwd_us"] = bench(lambda: torch.autograd.grad(sd(), (q, k, v), g))
# LayerNorm tail
y = torch.randn(T, H, device=dev).bfloat16()
r = torch.randn(T, H, device=dev).bfloat16()
gam = torch.ones(H, device=dev).bfloat16()
bet = torch.zeros(H, device=dev).bfloat16()
z, o2 = torch.empty_like(y), torch.empty_like(y)
mean, rstd = torch.empty(T, device=dev), torch.empty(T, device=dev)
dg, db, dbi = torch.zeros(H, device=dev), torch.zeros(H, device=dev), torch.zeros(H, device=dev)
for p in (0.0, 0.1):
    t = bench(lambda: C_.ln_fwd(y, r, gam, bet, z, o2, mean, rstd, 1e-12, p, 5))
    res[f"ln_fwd_p{p}_us"] = t
    res[f"ln_fwd_p{p}_TBs"] = 4 * T * H * 2 / t / 1e6
    dz, dy = torch.empty_like(y), torch.empty_like(y)
    t = bench(lambda: C_.ln_bwd(o2, z, mean, rstd, gam, dz, dy, None, dg, db, dbi, p, 5))
    res[f"ln_bwd_p{p}_us"] = t
    res[f"ln_bwd_p{p}_TBs"] = 4 * T * H * 2 / t / 1e6
a = torch.randn(T, I, device=dev).bfloat16()
gg = torch.empty_like(a)
t = bench(lambda: C_.gelu_fwd(a, gg)); res["gelu_fwd_us"] = t; res["gelu_fwd_TBs"] = 2 * T * I * 2 / t / 1e6
dbias = torch.zeros(I, device=dev)
t = bench(lambda: C_.gelu_bwd_colsum(gg, a, gg, dbias)); res["gelu_bwd_colsum_us"] = t
res["gelu_bwd_colsum_TBs"] = 3 * T * I * 2 / t / 1e6
t = bench(lambda: C_.colsum(a, dbias)); res["colsum_us"] = t; res["colsum_TBs"] = T * I * 2 / t / 1e6
res = {k: round(v, 2) for k, v in res.items()}
print(json.dumps(res, indent=1))
json.dump(res, open("gpurun_out/bench_ops.json", "w"), indent=1)
