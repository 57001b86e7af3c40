"""Epilogue store form (HSD_G2_NT: 0 plain global, 1 nt global, 2 buffer, 3 buffer sc1 (write-through), 4 buffer nt,
5 buffer sc0 sc1, 6 buffer nt sc1) on T x 3072 x K NT GEMMs (K = 64: epilogue-bound; K = 768: the FFN1 shape) and the
headline NT GEMMs; outputs must be bit-identical across forms.   python tools/store_policy_probe.py -> JSON lines"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from huggingface_sagemaker_tensorflow_distributed_amd.ops import hip  # noqa: E402

C_ = hip._C
dev = "cuda"
T = 131072
POLS = os.environ.get("POLS", "0,1,2,3,4,5,6").split(",")
rnd = lambda *s: (torch.rand(*s, device=dev) * 2 - 1).bfloat16()  # noqa: E731


def timeit(fn, iters=6):
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    st.record()
    for _ in range(iters):
        fn()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / iters * 1e3


for (N, K, epi) in [(3072, 64, 0), (3072, 64, 8), (3072, 768, 0), (3072, 768, 8), (3072, 768, 9), (2304, 768, 1),
                    (768, 768, 3), (768, 768, 0), (768, 3072, 4)]:
    a, b, bias, aux = rnd(T, K), rnd(N, K) * 0.05, rnd(N), rnd(T, N)
    c, c2 = torch.empty(T, N, device=dev, dtype=torch.bfloat16), torch.empty(T, N, device=dev, dtype=torch.bfloat16)
    db = torch.zeros(N, device=dev) if epi in (5, 9) else None

    def fn():
        C_.gemm2(a, b, c, 0, 0, epi, bias if epi in (1, 2, 3, 8) else None, aux if epi in (3, 4, 5, 9) else None,
                 c2 if epi in (2, 8) else None, 0.1 if epi == 3 else 0.0, 7, 1, None, db)

    r, ref, same = {p: [] for p in POLS}, None, True
    for rnd_i in range(3):
        for pol in POLS:
            os.environ["HSD_G2_NT"] = pol
            hip._C.refresh_env()  # launch knobs are cached (common.h HSD_KNOB)
            if rnd_i == 0:
                fn()
                torch.cuda.synchronize()
                if ref is None:
                    ref = c.clone()
                else:
                    same = same and torch.equal(ref, c)
            r[pol].append(timeit(fn))
    os.environ.pop("HSD_G2_NT")
    hip._C.refresh_env()  # launch knobs are cached (common.h HSD_KNOB)
    print(json.dumps({"N": N, "K": K, "epi": epi, "same": same, **{f"pol{p}": round(min(v), 1) for p, v in r.items()}}),
          flush=True)
