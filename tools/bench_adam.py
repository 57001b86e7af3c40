"""Fused Adam over a bert-base-sized flat store (109.5M fp32 params): unroll variants (HSD_ADAM_UNROLL), interleaved
rounds in one process, results checked bit-equal across variants.   python tools/bench_adam.py -> gpurun_out/bench_adam.json"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from huggingface_sagemaker_tensorflow_distributed_amd.ops import hip  # noqa: E402

n = 109_483_778 // 1024 * 1024 + 1024
dev = "cuda"
g0 = torch.randn(n, device=dev) * 1e-3
p0, m0, v0 = torch.randn(n, device=dev), torch.randn(n, device=dev) * 1e-3, torch.rand(n, device=dev) * 1e-6


def run(u, iters):
    os.environ["HSD_ADAM_UNROLL"] = str(u)
    hip._C.refresh_env()  # launch knobs are cached (common.h HSD_KNOB)
    p, m, v, out = p0.clone(), m0.clone(), v0.clone(), torch.empty(n, device=dev, dtype=torch.bfloat16)
    hip.adam_step(p, m, v, g0, out, None, 1e-4, 1e-7, 0.9, 0.999, 1.0, 0.0)
    torch.cuda.synchronize()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(iters):
        hip.adam_step(p, m, v, g0, out, None, 1e-4, 1e-7, 0.9, 0.999, 1.0, 0.0)
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / iters * 1e3, (p, m, v, out)


res, ref = {}, None
for rnd in range(3):
    for u in (1, 2, 4):
        us, outs = run(u, 10)
        res.setdefault(f"U{u}_us", []).append(round(us, 1))
        if u == 1 and ref is None:
            ref = outs
        elif rnd == 0:
            res[f"U{u}_same"] = all(torch.equal(a, b) for a, b in zip(outs, ref))
bytes_ = n * (4 * 4 + 3 * 4 + 2)
for u in (1, 2, 4):
    best = min(res[f"U{u}_us"])
    res[f"U{u}_TBs"] = round(bytes_ / best / 1e6, 2)
print(json.dumps(res))
os.makedirs("gpurun_out", exist_ok=True)
json.dump(res, open("gpurun_out/bench_adam.json", "w"), indent=1)
