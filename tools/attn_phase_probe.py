"""Phase timeline of the S=128 attention backward (attention128.hip, diagnostic stamps via _C.attn128_set_diag):
per-workgroup cycles spent loading operands, on the delta pre-pass, in the 4-block main loop, storing dK / dV, and on
dQ + its store; the in-kernel clock; how many workgroups run at once.  python tools/attn_phase_probe.py [p] [B]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from huggingface_sagemaker_tensorflow_distributed_amd.ops import hip  # noqa: E402

C_ = hip._C
dev = "cuda"
p = float(sys.argv[1]) if len(sys.argv) > 1 else 0.1
B = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
S, heads = 128, 12
H = heads * 64
T = B * S
torch.manual_seed(0)
qkv = torch.randn(T, 3 * H, device=dev).bfloat16()
out = torch.empty(T, H, device=dev, dtype=torch.bfloat16)
lse = torch.empty(B * heads * S, device=dev)
dqkv = torch.empty_like(qkv)
dout = torch.randn(T, H, device=dev).bfloat16()
mask = torch.zeros(B, S, device=dev)
dbias = torch.zeros(3 * H, device=dev)
km = hip._keep_mask(B, S, heads, p, dev) if os.environ.get("ATTN_KMASK", "1") == "1" else None
C_.attn_fwd(qkv, mask, out, lse, B, S, heads, p, 123, km)
diag = torch.zeros(B * heads * 8, dtype=torch.int64, device=dev)
for _ in range(3):
    C_.attn_bwd(qkv, mask, out, dout, lse, dqkv, None, B, S, heads, p, 123, dbias, km)
C_.attn128_set_diag(diag)
C_.attn_bwd(qkv, mask, out, dout, lse, dqkv, None, B, S, heads, p, 123, dbias, km)
torch.cuda.synchronize()
C_.attn128_set_diag(None)
d = diag.view(-1, 8).cpu().double()
ph = d[:, 1:6] - d[:, 0:5]
names = ["load", "delta", "loop", "dkdv_store", "dq"]
tot = d[:, 5] - d[:, 0]
clk = (tot / ((d[:, 7] - d[:, 6]) / 100.0)).median().item() / 1e3  # memtime ticks per us / 1000 = GHz
res = {"p": p, "B": B, "clock_ghz": round(clk, 3), "wg_cycles_median": int(tot.median()),
       **{f"{n}_median": int(ph[:, i].median()) for i, n in enumerate(names)},
       **{f"{n}_p90": int(ph[:, i].quantile(0.9)) for i, n in enumerate(names)}}
# concurrency: workgroups alive at the median workgroup's midpoint (real-time stamps, 100 MHz)
s0, s1 = d[:, 6], d[:, 7]
span_us = (s1.max() - s0.min()).item() / 100.0
res["kernel_span_us"] = round(span_us, 1)
res["wg_lifetime_us_median"] = round(((s1 - s0).median() / 100.0).item(), 2)
res["avg_wgs_in_flight"] = round(((s1 - s0).sum() / (s1.max() - s0.min())).item(), 1)
print(json.dumps(res))
