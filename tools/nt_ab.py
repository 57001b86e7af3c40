"""A/B of the NT GEMM path choice (gemm2 256 x 256 tiles / split-K slabs / gemm2s 128 x 128 tiles at 2 or 3 LDS
stages) over the BERT layer's NT GEMMs (base and large widths, the epilogues the step uses) and token counts,
interleaved rounds in one process.
    python tools/nt_ab.py "HSD_G2_SMALL=0" "HSD_G2_SMALL=1 HSD_G2S_STAGES=2" ...  -> one JSON line per case"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from huggingface_sagemaker_tensorflow_distributed_amd.ops import hip  # noqa: E402

C_ = hip._C
dev = "cuda"
SETTINGS = sys.argv[1:]
TOKENS = [int(t) for t in os.environ.get("NT_T", "4096,8192,16384,32768").split(",")]
SHAPES = []
for H in (768, 1024):
    I = 4 * H
    SHAPES += [(3 * H, H, 1), (H, H, 3), (I, H, 8), (H, I, 3), (I, H, 9), (H, I, 4), (H, H, 0), (H, 3 * H, 4)]


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


rnd = lambda *s: (torch.rand(*s, device=dev) * 2 - 1).bfloat16()  # noqa: E731
for T in TOKENS:
    for N, K, epi in SHAPES:
        a, b, bias, aux = rnd(T, K), rnd(N, K) * 0.05, rnd(N), rnd(T, N)
        c = torch.empty(T, N, device=dev, dtype=torch.bfloat16)
        c2 = torch.empty_like(c) if epi in (2, 8) else None
        db = torch.zeros(N, device=dev) if epi in (5, 9) else None
        t = {s: [] for s in SETTINGS}
        for _ in range(3):
            for s in SETTINGS:
                apply(s)
                t[s].append(timeit(lambda: C_.gemm2(a, b, c, 0, 0, epi, bias if epi in (1, 2, 3, 8) else None,
                                                    aux if epi in (3, 4, 5, 9) else None, c2,
                                                    0.1 if epi == 3 else 0.0, 7, 0, None, db)))
                clear(s)
        fl = 2.0 * T * N * K
        print(json.dumps({"T": T, "N": N, "K": K, "epi": epi,
                          **{f"[{s}]": f"{min(v):.1f}us {fl / min(v) / 1e6:.0f}TF" for s, v in t.items()}}), flush=True)
