"""Runs the attention forward and backward `iters` times (for rocprofv3 --pmc passes); prints the mean times of
both directions at p = 0 and p = 0.1. Default shape: BERT-base B=1024 S=128; ATTN_SHAPE=B,S,heads overrides
(bert-large S=512: ATTN_SHAPE=64,512,16)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from huggingface_sagemaker_tensorflow_distributed_amd.ops import hip  # noqa: E402

C_ = hip._C
dev = "cuda"
B, S, heads = (int(v) for v in os.environ.get("ATTN_SHAPE", "1024,128,12").split(","))
H = heads * 64
T = B * S
p = float(sys.argv[1]) if len(sys.argv) > 1 else 0.1
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 5
torch.manual_seed(0)
qkv = torch.randn(T, 3 * H, device=dev).bfloat16()
out = torch.empty(T, H, device=dev, dtype=torch.bfloat16)
lse = torch.empty(B * heads * S, device=dev)
dqkv = torch.empty_like(qkv)
dout = torch.randn(T, H, device=dev).bfloat16()
mask = torch.zeros(B, S, device=dev)
dbias = torch.zeros(3 * H, device=dev)
ws = torch.empty(B * heads * S, device=dev) if S > 128 else None  # delta workspace of the streaming kernels
st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
# the production path: the S = 128 forward writes its dropout keep bits for the backward (ops/hip.py _keep_mask);
# ATTN_KMASK=0 times the re-hashing backward instead
use_km = os.environ.get("ATTN_KMASK", "1") == "1"
for pp in sorted({0.0, p}):
    km = hip._keep_mask(B, S, heads, pp, dev) if use_km else None
    C_.attn_fwd(qkv, mask, out, lse, B, S, heads, pp, 123, km)
    torch.cuda.synchronize()
    st.record()
    for _ in range(iters):
        C_.attn_fwd(qkv, mask, out, lse, B, S, heads, pp, 123, km)
    en.record()
    torch.cuda.synchronize()
    f = st.elapsed_time(en) / iters * 1e3
    st.record()
    for _ in range(iters):
        C_.attn_bwd(qkv, mask, out, dout, lse, dqkv, ws, B, S, heads, pp, 123, dbias, km)
    en.record()
    torch.cuda.synchronize()
    b = st.elapsed_time(en) / iters * 1e3
    print(f"p={pp} kmask={km is not None}: fwd {f:.1f} us  bwd {b:.1f} us", flush=True)
