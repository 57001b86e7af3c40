"""A/B of the TT weight-gradient GEMM path (g.buf[N, K] += dyᵀ x, split-K slabs + reduce included) over BERT
weight shapes and token counts, interleaved rounds in one process.
    python tools/wgrad_ab.py "HSD_G2_SMALL_TT=0" "HSD_G2_SMALL_TT=1 HSD_G2S_STAGES=4" ...  -> one JSON line per case"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from huggingface_sagemaker_tensorflow_distributed_amd.ops import hip  # noqa: E402

C_ = hip._C
dev = "cuda"
SETTINGS = sys.argv[1:]
SHAPES = [(2304, 768), (768, 768), (3072, 768), (768, 3072), (3072, 1024), (1024, 1024), (4096, 1024), (1024, 4096)]
TOKENS = [int(t) for t in os.environ.get("WGRAD_T", "4096,8192,16384").split(",")]


def apply(setting):
    for kv in setting.split():
        k, v = kv.split("=")
        os.environ[k] = v
        hip._C.refresh_env()  # launch knobs are cached (common.h HSD_KNOB)


def clear(setting):
    for kv in setting.split():
        os.environ.pop(kv.split("=")[0], None)
        hip._C.refresh_env()  # launch knobs are cached (common.h HSD_KNOB)


def timeit(fn, iters=10):
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    st.record()
    for _ in range(iters):
        fn()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / iters * 1e3


for T in TOKENS:
    for N, K in SHAPES:
        dy = (torch.rand(T, N, device=dev) * 2 - 1).bfloat16()
        x = (torch.rand(T, K, device=dev) * 2 - 1).bfloat16()
        g = torch.zeros(N, K, device=dev)
        t = {s: [] for s in SETTINGS}
        sps = {}
        for _ in range(3):
            for s in SETTINGS:
                apply(s)
                sp = C_.gemm2_splits(N, K, T)
                sps[s] = sp
                ws = torch.empty(sp * N * K, device=dev)
                t[s].append(timeit(lambda: C_.gemm2(dy, x, g, 1, 1, 7, None, None, None, 0.0, 0, sp, ws, None)))
                clear(s)
        fl = 2.0 * T * N * K
        print(json.dumps({"T": T, "N": N, "K": K, **{f"[{s}]": f"{min(v):.1f}us {fl / min(v) / 1e6:.0f}TF sp{sps[s]}"
                                                     for s, v in t.items()}}), flush=True)
