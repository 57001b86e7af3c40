"""Embedding backward time vs HSD_EMBED_BWD_BLOCKS (target block count) at the headline and the
reference's per-rank shapes.   python tools/embed_bwd_probe.py  -> one line per (shape, knob)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from huggingface_sagemaker_tensorflow_distributed_amd.ops import hip  # noqa: E402

C_ = hip._C
dev = "cuda"
V = 30522


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


for B, S, H in ((1024, 128, 768), (8, 512, 1024), (32, 128, 768), (64, 512, 1024)):
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
    mean, rstd = torch.empty(B * S, device=dev), torch.empty(B * S, device=dev)
    C_.embed_fwd(ids, pos, tt, word, pw, tw, g, be, out, mean, rstd, 1e-12, 0.1, 5)
    dout = torch.randn(B * S, H, device=dev).bfloat16()
    ref = None
    for rows in (2048, 1024, 512, 256):
        os.environ["HSD_EMBED_BWD_BLOCKS"] = str(rows)
        C_.refresh_env()
        gs = [torch.zeros(V, H, device=dev), torch.zeros(512, H, device=dev), torch.zeros(2, H, device=dev),
              torch.zeros(H, device=dev), torch.zeros(H, device=dev)]
        fn = lambda: C_.embed_bwd(dout, ids, pos, tt, word, pw, tw, g, mean, rstd, *gs, B, S, True, 0.1, 5)  # noqa: E731
        for t in gs:
            t.zero_()
        fn()
        torch.cuda.synchronize()
        got = [t.clone() for t in gs]
        if ref is None:
            ref = got
        err = max(float((a - b).abs().max() / (b.abs().max() + 1e-30)) for a, b in zip(got, ref))
        us = sorted(timeit(fn) for _ in range(3))[1]
        print(f"B={B} S={S} H={H} blocks~{rows}: {us:.1f} us  max rel diff vs 2048 {err:.1e}", flush=True)
