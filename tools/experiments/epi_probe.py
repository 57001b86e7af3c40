"""Fused-epilogue NT GEMMs of the BERT-base B=1024 step under several main-loop schedules (HSD_G2_SYNC),
interleaved rounds in one process: does a persistent kernel (3: next tile's DMA and MFMAs under the epilogue's
store drain) pay for the store-heavy epilogues?   python tools/epi_probe.py [T] -> gpurun_out/epi_probe.json"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from huggingface_sagemaker_tensorflow_distributed_amd.ops import hip  # noqa: E402

C_ = hip._C
T = int(sys.argv[1]) if len(sys.argv) > 1 else 131072
VARS = [int(v) for v in os.environ.get("PROBE_SYNC", "1,3,4").split(",")]
dev = "cuda"


def rnd(*s):
    return (torch.rand(*s, device=dev) * 2 - 1).bfloat16()


def timeit(fn, iters=10):
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    st.record()
    for _ in range(iters):
        fn()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / iters * 1e-3


H, I = 768, 3072
x, w1, b1 = rnd(T, H), rnd(I, H), rnd(I)
act, pre = torch.empty(T, I, device=dev, dtype=torch.bfloat16), torch.empty(T, I, device=dev, dtype=torch.bfloat16)
w2, b2, res = rnd(H, I), rnd(H), rnd(T, H)
z = torch.empty(T, H, device=dev, dtype=torch.bfloat16)
dy, w2t, aux = rnd(T, H), rnd(I, H), rnd(T, I)
da = torch.empty(T, I, device=dev, dtype=torch.bfloat16)
db = torch.zeros(I, device=dev)
w1t, dz = rnd(H, I), rnd(T, H)
dh = torch.empty(T, H, device=dev, dtype=torch.bfloat16)
cases = {
    "ffn1_fwd_gelu_d(E8)": (2 * T * I * H, lambda: C_.gemm2(x, w1, pre, 0, 0, 8, b1, None, act, 0.0, 0, 1, None, None)),
    "ffn2_fwd_drop_res(E3)": (2 * T * H * I, lambda: C_.gemm2(act, w2, z, 0, 0, 3, b2, res, None, 0.1, 7, 1, None, None)),
    "ffn2_dgrad_mul_dbias(E9)": (2 * T * I * H, lambda: C_.gemm2(dy, w2t, da, 0, 0, 9, None, aux, None, 0.0, 0, 1, None, db)),
    "ffn1_dgrad_res(E4)": (2 * T * H * I, lambda: C_.gemm2(da, w1t, dh, 0, 0, 4, None, dz, None, 0.0, 0, 1, None, None)),
}
res_t = {k: {} for k in cases}
for r in range(3):
    for k, (fl, fn) in cases.items():
        for v in VARS:
            os.environ["HSD_G2_SYNC"] = str(v)
            hip._C.refresh_env()  # launch knobs are cached (common.h HSD_KNOB)
            res_t[k].setdefault(f"s{v}", []).append(fl / timeit(fn) / 1e12)
        os.environ.pop("HSD_G2_SYNC", None)
        hip._C.refresh_env()  # launch knobs are cached (common.h HSD_KNOB)
out = {k: {kk: round(sorted(vv)[1], 1) for kk, vv in v.items()} for k, v in res_t.items()}
for k, v in out.items():
    print(k, v, flush=True)
os.makedirs("gpurun_out", exist_ok=True)
json.dump(out, open("gpurun_out/epi_probe.json", "w"), indent=1)
