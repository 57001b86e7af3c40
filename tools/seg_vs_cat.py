"""Segmented-K split-product GEMM (gemm2_seg over hi / lo halves) vs the same GEMM over three-block concatenated copies
(gemm2_f32nt / gemm2 TT on split3 outputs), timed in one process, interleaved rounds: the fp32 step's shapes at
bert-large B = 8 S = 512 (T = 4,096 tokens).     python tools/seg_vs_cat.py [T]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from huggingface_sagemaker_tensorflow_distributed_amd.ops import hip32 as h  # noqa: E402

C_ = h._C
dev = "cuda"
T = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
SHAPES = [(1024, 3072), (1024, 1024), (1024, 4096), (4096, 1024)]  # (K_in, N_out) of the four linears


def timed(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / n


for K, N in SHAPES:
    torch.manual_seed(K + N)
    x, w, dy = torch.randn(T, K, device=dev), torch.randn(N, K, device=dev) * 0.05, torch.randn(T, N, device=dev)
    xh, xl = h._split2(x)
    wh, wl = h._split2(w)
    dh, dl = h._split2(dy)
    xc, wc = h._split(x, h.PAT_A), h._split(w, h.PAT_B)
    dc, wr = h._split(dy, h.PAT_A), h._split(w, h.PAT_B, rows=True)
    dr, xr = h._split(dy, h.PAT_A, rows=True), h._split(x, h.PAT_B, rows=True)
    y = torch.empty(T, N, device=dev)
    dx = torch.empty(T, K, device=dev)
    g = torch.zeros(N, K, device=dev)
    sp = C_.gemm2_splits(N, K, 3 * T)
    ws = torch.empty(max(1, sp) * N * K, device=dev)
    # the halves as the two planes of one allocation (hi at +0, lo at +T·K) rather than two allocations
    one = torch.empty(2, *x.shape, dtype=torch.bfloat16, device=dev)
    one[0].copy_(xh)
    one[1].copy_(xl)
    onew = torch.empty(2, *w.shape, dtype=torch.bfloat16, device=dev)
    onew[0].copy_(wh)
    onew[1].copy_(wl)
    cases = {
        "fwd_seg_1buf": lambda: C_.gemm2_seg([one[0], one[0], one[1]], [onew[0], onew[1], onew[0]], y, 0, 0),
        "fwd_seg_order": lambda: C_.gemm2_seg([xh, xl, xh], [wh, wh, wl], y, 0, 0),
        "fwd_seg": lambda: C_.gemm2_seg([xh, xh, xl], [wh, wl, wh], y, 0, 0),
        "fwd_cat": lambda: C_.gemm2_f32nt(xc, wc, y, 0),
        "dgrad_seg": lambda: C_.gemm2_seg([dh, dh, dl], [wh, wl, wh], dx, 0, 1),
        "dgrad_cat": lambda: C_.gemm2_f32nt(dc, wr, dx, 1),
        "wgrad_seg": lambda: C_.gemm2_seg([dh, dh, dl], [xh, xl, xh], g, 1, 1),
        "wgrad_cat": lambda: C_.gemm2(dr, xr, g, 1, 1, 7, None, None, None, 0.0, 0, sp, ws, None, None, 0),
    }
    # the NT segmented GEMMs again on 256 x 256 tiles split over K into slabs (HSD_SEG_NT_SMALL=0) where the default
    # takes 128 x 128 tiles
    cases["fwd_seg_slab"], cases["dgrad_seg_slab"] = cases["fwd_seg"], cases["dgrad_seg"]
    res = {k: [] for k in cases}
    for _ in range(3):
        for k, fn in cases.items():
            os.environ["HSD_SEG_NT_SMALL"] = "0" if k.endswith("_slab") else "1"
            C_.refresh_env()
            res[k].append(timed(fn))
    os.environ.pop("HSD_SEG_NT_SMALL")
    C_.refresh_env()
    print(json.dumps({"T": T, "K": K, "N": N, **{k: round(min(v), 1) for k, v in res.items()}}), flush=True)
