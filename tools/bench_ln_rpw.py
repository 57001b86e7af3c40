"""Plain LayerNorm forward (the encoder's LN after the fused GEMM epilogue) at T x 768 for several rows-per-wave
(HSD_LN_FWD_RPW), interleaved rounds in one process.   python tools/bench_ln_rpw.py [T]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from huggingface_sagemaker_tensorflow_distributed_amd.ops import hip  # noqa: E402

C_ = hip._C
dev = "cuda"
T = int(sys.argv[1]) if len(sys.argv) > 1 else 131072
H = 768
y = torch.randn(T, H, device=dev).bfloat16()
g = (torch.rand(H, device=dev) + 0.5).bfloat16()
b = torch.randn(H, device=dev).bfloat16()
o = torch.empty_like(y)
mean = torch.empty(T, device=dev)
rstd = torch.empty(T, device=dev)


def run():
    C_.ln_fwd(y, None, g, b, None, o, mean, rstd, 1e-12, 0.0, 0)


def timeit(iters=30):
    run()
    torch.cuda.synchronize()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(iters):
        run()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / iters * 1e3


modes = ["0", "2", "4", "6", "8", "12", "16"]
t = {m: [] for m in modes}
for _ in range(4):
    for m in modes:
        os.environ["HSD_LN_FWD_RPW"] = m
        hip._C.refresh_env()  # launch knobs are cached (common.h HSD_KNOB)
        t[m].append(timeit())
res = {f"rpw{m}_us": round(min(v), 1) for m, v in t.items()}
res.update({f"rpw{m}_TBs": round(2 * T * H * 2 / (min(v) * 1e-6) / 1e12, 2) for m, v in t.items()})
print(json.dumps(res))
