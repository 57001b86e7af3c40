"""Persistent GEMMs under co-running CU holders: static vs dynamic tile walk (VERDICT r3 'Next round' item 2).

A data-parallel rank runs RCCL all-reduce kernels (one workgroup per channel, each holding a CU) beside its backward
GEMMs. A persistent GEMM workgroup whose CU is held starts late; with the static tile walk it still owns 1/grid of the
tiles, so the GEMM ends late by the hold time. With the dynamic tile queue (gemm_common.h tq_*), the others take its
tiles. This measures both on one GPU with the cu_hog kernel (elementwise.hip: k workgroups x 160 KiB LDS, one per CU,
for `us` microseconds) launched on a side stream right before each GEMM.

    python tools/contention_ab.py [T] [us]  -> JSON lines: shape, k, static / dynamic us, proportional bound
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from huggingface_sagemaker_tensorflow_distributed_amd.ops import hip  # noqa: E402

C_ = hip._C
dev = "cuda"
T = int(sys.argv[1]) if len(sys.argv) > 1 else 131072
HOLD = float(sys.argv[2]) if len(sys.argv) > 2 else 400.0
rnd = lambda *s: (torch.rand(*s, device=dev) * 2 - 1).bfloat16()  # noqa: E731
side = torch.cuda.Stream()
# (name, N, K, epi): FFN1 forward (GELU + GELU'), FFN2 dgrad (x GELU', bias-gradient sums), QKV forward
SHAPES = [("ffn1_fwd", 3072, 768, 8), ("ffn2_dgrad", 3072, 768, 9), ("qkv_fwd", 2304, 768, 1)]


def run(a, b, c, c2, bias, aux, db, epi, k, reps=6):
    cur = torch.cuda.current_stream()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(reps):
        side.wait_stream(cur)
        cur.synchronize()
        if k:
            with torch.cuda.stream(side):
                C_.cu_hog(k, HOLD)
        st.record()
        C_.gemm2(a, b, c, 0, 0, epi, bias if epi in (1, 8) else None, aux if epi == 9 else None, c2, 0.0, 7, 1,
                 None, db)
        en.record()
        torch.cuda.synchronize()
        ts.append(st.elapsed_time(en) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


for name, N, K, epi in SHAPES:
    a, b = rnd(T, K), rnd(N, K) * 0.05
    bias, aux = rnd(N), rnd(T, N)
    c = torch.empty(T, N, device=dev, dtype=torch.bfloat16)
    c2 = torch.empty_like(c) if epi == 8 else None
    db = torch.zeros(N, device=dev) if epi == 9 else None
    outs = {}
    res = {}
    for k in (0, 14, 28, 56):
        for dyn in ("0", "1"):
            os.environ["HSD_G2_DYN"] = dyn
            C_.refresh_env()
            res[(k, dyn)] = run(a, b, c, c2, bias, aux, db, epi, k)
            if k == 0:
                outs[dyn] = c.clone()
    os.environ.pop("HSD_G2_DYN", None)
    C_.refresh_env()
    same = torch.equal(outs["0"], outs["1"])
    base = res[(0, "1")]
    for k in (0, 14, 28, 56):
        print(json.dumps({"gemm": name, "T": T, "hold_us": HOLD, "k_cus": k, "static_us": round(res[(k, "0")], 1),
                          "dynamic_us": round(res[(k, "1")], 1),
                          "proportional_us": round(base + k * HOLD / 256.0, 1) if k else round(base, 1),
                          "bit_identical": same}), flush=True)
