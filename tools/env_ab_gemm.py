"""A/B an environment switch of the NT GEMM path on the headline layer's NT GEMMs (tools/gemm_sol.py shapes, the
epilogues the step uses), interleaved rounds in one process; outputs must be bit-identical across settings.
    python tools/env_ab_gemm.py HSD_G2_AUX_PF 0,1 [T]  -> one JSON line per GEMM"""
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
VAR = sys.argv[1]
VALS = sys.argv[2].split(",")
T = int(sys.argv[3]) if len(sys.argv) > 3 else 131072
rnd = lambda *s: (torch.rand(*s, device=dev) * 2 - 1).bfloat16()  # noqa: E731


def timeit(fn, iters=8):
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    st.record()
    for _ in range(iters):
        fn()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / iters * 1e3


for name, lay, M, N, K, epi in GEMMS:
    if lay != "NT":
        continue
    M = T
    a, b = rnd(M, K), rnd(N, K) * 0.05
    bias, aux = rnd(N), rnd(M, N)
    outs = {}
    t = {v: [] for v in VALS}
    for rnd_i in range(3):
        for v in VALS:
            os.environ[VAR] = v
            hip._C.refresh_env()  # launch knobs are cached (common.h HSD_KNOB)
            c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            c2 = torch.empty_like(c) if epi in (2, 8) else None
            db = torch.zeros(N, device=dev) if epi in (5, 9) else None

            def fn():
                C_.gemm2(a, b, c, 0, 0, epi, bias if epi in (1, 2, 3, 8) else None,
                         aux if epi in (3, 4, 5, 9) else None, c2, 0.1 if epi == 3 else 0.0, 7, 1, None, db)

            if rnd_i == 0:
                fn()
                torch.cuda.synchronize()
                outs[v] = c.clone()
            t[v].append(timeit(fn))
    os.environ.pop(VAR, None)
    hip._C.refresh_env()  # launch knobs are cached (common.h HSD_KNOB)
    same = all(torch.equal(outs[VALS[0]], outs[v]) for v in VALS[1:])
    print(json.dumps({"gemm": name, "epi": epi, "same": same, **{f"{VAR}={v}": round(min(t[v]), 1) for v in VALS}}),
          flush=True)
