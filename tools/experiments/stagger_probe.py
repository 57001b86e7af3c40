"""Epilogue write-burst probe: time the headline NT GEMMs with the CU-group phase stagger (HSD_G2_STAGGER sleep
iterations of 1,024 cycles for every second CU's first workgroup) at several values, interleaved rounds in one
process.   python tools/stagger_probe.py [values] -> gpurun_out/stagger_probe.json"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from huggingface_sagemaker_tensorflow_distributed_amd.ops import hip  # noqa: E402
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tools"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tools"))
from gemm_sol import GEMMS  # noqa: E402

C_ = hip._C
dev = "cuda"
VALS = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "0,8,16,24,36,48,72").split(",")]
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


res = {}
for name, lay, M, N, K, epi in GEMMS:
    if lay != "NT":
        continue
    a, b = rnd(M, K), rnd(N, K) * 0.05
    bias, aux = rnd(N), rnd(M, N)
    c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    c2 = torch.empty_like(c) if epi in (2, 8) else None
    db = torch.zeros(N, device=dev) if epi in (5, 9) else None

    def fn():
        C_.gemm2(a, b, c, 0, 0, epi, bias if epi in (1, 2, 3, 8) else None, aux if epi in (3, 4, 5, 9) else None, c2,
                 0.1 if epi == 3 else 0.0, 7, 1, None, db)

    t = {v: [] for v in VALS}
    for _ in range(3):
        for v in VALS:
            os.environ["HSD_G2_STAGGER"] = str(v)
            t[v].append(timeit(fn))
    os.environ["HSD_G2_STAGGER"] = "0"
    res[name] = {str(v): round(min(t[v]), 1) for v in VALS}
    print(name, res[name], flush=True)
os.makedirs("gpurun_out", exist_ok=True)
json.dump(res, open("gpurun_out/stagger_probe.json", "w"), indent=1)
