"""One-off probe: torch/hipBLASLt GEMM rates on BERT-base shapes and HF eager BERT step time.

Used to set the yardstick our kernels must beat (results copied into profiles/).
"""
import json, time, sys
import torch

dev = "cuda"
res = {}
def bench(fn, iters=20, warm=5):
    for _ in range(warm): fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters): fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters

T = 32768
shapes = {"qkv": (T, 2304, 768), "out": (T, 768, 768), "ffn1": (T, 3072, 768), "ffn2": (T, 768, 3072)}
for name, (M, N, K) in shapes.items():
    a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=dev, dtype=torch.bfloat16)
    dy = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
    fl = 2 * M * N * K
    t_f = bench(lambda: a @ w.t())
    t_d = bench(lambda: dy @ w)
    t_w = bench(lambda: dy.t() @ a)
    res[name] = {"fwd_TF": fl / t_f / 1e12, "dgrad_TF": fl / t_d / 1e12, "wgrad_TF": fl / t_w / 1e12,
                 "fwd_ms": t_f * 1e3}
    print(name, res[name], flush=True)

# elementwise bandwidth (LayerNorm, gelu)
x = torch.randn(T, 768, device=dev, dtype=torch.bfloat16)
ln = torch.nn.LayerNorm(768).to(dev, torch.bfloat16)
t = bench(lambda: ln(x)); res["torch_ln_GBs"] = 2 * x.numel() * 2 / t / 1e9
h = torch.randn(T, 3072, device=dev, dtype=torch.bfloat16)
t = bench(lambda: torch.nn.functional.gelu(h)); res["torch_gelu_GBs"] = 2 * h.numel() * 2 / t / 1e9
print(res, flush=True)

# HF eager bert-base step
from transformers import BertConfig, BertForSequenceClassification
cfg = BertConfig()
for B in (64, 256):
    model = BertForSequenceClassification(cfg).to(dev)
    opt = torch.optim.AdamW(model.parameters(), lr=1e-5, fused=True)
    ids = torch.randint(0, 30522, (B, 128), device=dev)
    am = torch.ones(B, 128, device=dev, dtype=torch.long)
    lab = torch.randint(0, 2, (B,), device=dev)
    def step():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = model(input_ids=ids, attention_mask=am, labels=lab)
        out.loss.backward()
        opt.step(); opt.zero_grad(set_to_none=True)
    t = bench(step, iters=10, warm=3)
    res[f"hf_eager_amp_B{B}_seq_s"] = B / t
    print(B, B / t, flush=True)
    del model, opt
json.dump(res, open("gpurun_out/probe_baseline.json", "w"), indent=1)
