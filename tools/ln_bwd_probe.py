"""LayerNorm backward (ln_bwd_fused_kernel, the production path: dropout, dz + dy, dgamma / dbeta / dbias) vs the
rows-per-wave floor HSD_LN_BWD_MIN_RPW at the headline and the reference's per-rank shapes.
    python tools/ln_bwd_probe.py   -> one line per (shape, floor): us, TB/s, max rel diff of dgamma vs the default"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from huggingface_sagemaker_tensorflow_distributed_amd.ops import hip  # noqa: E402

C_ = hip._C
dev = "cuda"


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


for T, H in ((4096, 1024), (4096, 768), (32768, 1024), (131072, 768)):
    torch.manual_seed(0)
    z = torch.randn(T, H, device=dev).bfloat16()
    dout = torch.randn(T, H, device=dev).bfloat16()
    g = (torch.rand(H, device=dev) + 0.5).bfloat16()
    mean, rstd = z.float().mean(1), torch.rsqrt(z.float().var(1, unbiased=False) + 1e-12)
    dz, dy = torch.empty_like(z), torch.empty_like(z)
    dg, db, dbias = torch.zeros(H, device=dev), torch.zeros(H, device=dev), torch.zeros(H, device=dev)
    fn = lambda: C_.ln_bwd(dout, z, mean, rstd, g, dz, dy, None, dg, db, dbias, 0.1, 7)  # noqa: E731
    ref = None
    for rpw in (4, 1, 2, 8, 16, 32):
        os.environ["HSD_LN_BWD_MIN_RPW"] = str(rpw)
        C_.refresh_env()
        dg.zero_()
        fn()
        torch.cuda.synchronize()
        got = dg.clone()
        if ref is None:
            ref = got
        err = float((got - ref).abs().max() / ref.abs().max())
        us = sorted(timeit(fn) for _ in range(3))[1]
        print(f"T={T} H={H} min_rpw={rpw}: {us:.1f} us {4 * T * H * 2 / us / 1e6:.2f} TB/s  dgamma rel diff {err:.1e}",
              flush=True)
