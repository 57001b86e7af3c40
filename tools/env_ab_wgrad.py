"""A/B an environment switch on the headline layer's TT weight-gradient GEMMs (tools/gemm_sol.py GEMMS, T tokens),
interleaved rounds in one process: one JSON line per GEMM with the best-of-3 time of each setting.
    python tools/env_ab_wgrad.py HSD_G2_SYNC 4,7 [T]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gemm_sol import GEMMS  # noqa: E402

from huggingface_sagemaker_tensorflow_distributed_amd.ops import hip  # noqa: E402

C_ = hip._C
dev = "cuda"
VAR, VALS = sys.argv[1], sys.argv[2].split(",")
T = int(sys.argv[3]) if len(sys.argv) > 3 else 131072
rnd = lambda *s: (torch.rand(*s, device=dev) * 2 - 1).bfloat16()  # noqa: E731


def timeit(fn, iters=5):
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    st.record()
    for _ in range(iters):
        fn()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / iters * 1e3


for name, lay, M, N, K, epi in GEMMS:
    if lay != "TT":
        continue
    K = T
    dy, x = rnd(K, M), rnd(K, N)
    t = {v: [] for v in VALS}
    outs = {}
    for r in range(3):
        for v in VALS:
            os.environ[VAR] = v
            C_.refresh_env()
            g = torch.zeros(M, N, device=dev)
            sp = C_.gemm2_splits(M, N, K)
            ws = torch.empty(sp * M * N, device=dev)

            def fn():
                C_.gemm2(dy, x, g, 1, 1, 7, None, None, None, 0.0, 0, sp, ws, None)

            if r == 0:
                g.zero_()
                fn()
                torch.cuda.synchronize()
                outs[v] = g.clone()
            t[v].append(timeit(fn))
    os.environ.pop(VAR, None)
    C_.refresh_env()
    same = all(torch.equal(outs[VALS[0]], outs[v]) for v in VALS[1:])
    flops = 2.0 * M * N * K
    print(json.dumps({"gemm": name, "M": M, "N": N, "K": K, "splits": C_.gemm2_splits(M, N, K), "same": same,
                      **{f"{VAR}={v}": round(min(t[v]), 1) for v in VALS},
                      **{f"TF@{v}": round(flops / min(t[v]) / 1e6, 0) for v in VALS}}), flush=True)
