"""gemm3 (two 4-wave workgroups per CU, 256 x 128 tiles) vs gemm2 (one 8-wave 256 x 256 workgroup per CU) on the
B = 1024 BERT-base step's GEMMs: every forward / dgrad epilogue the step uses and the four weight gradients.

    python tools/gemm3_probe.py [T]        -> gpurun_out/gemm3_probe.json

NT outputs must be BIT-identical between the two bodies (same K order: BK 64 = two 32-deep MFMA steps); TT
weight gradients use different split-K factors, so they are compared with an fp32 reference. Timings are
interleaved rounds in one process (cdna_hip_programming.md §5.4 rule 24), random operands.
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
ROUNDS = int(os.environ.get("ROUNDS", "3"))
MASK = os.environ.get("G3_MASK", "3")
torch.manual_seed(0)


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


def with_g3(on, fn):
    os.environ["HSD_GEMM3"] = MASK if on else "0"
    try:
        return fn()
    finally:
        os.environ["HSD_GEMM3"] = "0"


# name: (M, N, K, epi, bias, aux, two_out, p_drop, dbias)
NT = {
    "qkv_fwd_bias": (T, 2304, 768, 1, True, False, False, 0.0, False),
    "out_fwd_dropres": (T, 768, 768, 3, True, True, False, 0.1, False),
    "ffn1_fwd_gelu_d": (T, 3072, 768, 8, True, False, True, 0.0, False),
    "ffn2_fwd_dropres": (T, 768, 3072, 3, True, True, False, 0.1, False),
    "qkv_dgrad_res": (T, 768, 2304, 4, False, True, False, 0.0, False),
    "out_dgrad_store": (T, 768, 768, 0, False, False, False, 0.0, False),
    "ffn1_dgrad_res": (T, 768, 3072, 4, False, True, False, 0.0, False),
    "ffn2_dgrad_mul": (T, 3072, 768, 9, False, True, False, 0.0, True),
}
TT = {"qkv_wgrad": (2304, 768), "out_wgrad": (768, 768), "ffn1_wgrad": (3072, 768), "ffn2_wgrad": (768, 3072)}

cases = {}
out = {}
for name, (M, N, K, epi, has_b, has_aux, two, p, has_db) in NT.items():
    x, w = rnd(M, K), rnd(N, K)
    b = rnd(N) if has_b else None
    aux = rnd(M, N) if has_aux else None
    ys = [torch.empty(M, N, device=dev, dtype=torch.bfloat16) for _ in range(2)]
    y2s = [torch.empty(M, N, device=dev, dtype=torch.bfloat16) if two else None for _ in range(2)]
    dbs = [torch.zeros(N, device=dev) if has_db else None for _ in range(2)]

    def run(i, x=x, w=w, b=b, aux=aux, epi=epi, p=p, ys=ys, y2s=y2s, dbs=dbs):
        return C_.gemm2(x, w, ys[i], 0, 0, epi, b, aux, y2s[i], p, 1234, 1, None, dbs[i])

    with_g3(False, lambda: run(0))
    with_g3(True, lambda: run(1))
    torch.cuda.synchronize()
    rec = {"same_y": bool(torch.equal(ys[0], ys[1]))}
    if two:
        rec["same_y2"] = bool(torch.equal(y2s[0], y2s[1]))
    if has_db:
        rec["dbias_rel"] = ((dbs[0] - dbs[1]).abs().max() / dbs[0].abs().max()).item()
    ref = x[:256].float() @ w.float().t()
    if epi == 0:
        rec["err_ref"] = ((ys[1][:256].float() - ref).abs().max() / ref.abs().max()).item()
    out[name] = rec
    cases[name] = (2.0 * M * N * K, lambda run=run: run(0), lambda run=run: run(1))
    print("checked", name, rec, flush=True)

for name, (N, K) in TT.items():
    dy, x = rnd(T, N), rnd(T, K)
    gws = [torch.zeros(N, K, device=dev) for _ in range(2)]
    os.environ["HSD_GEMM3"] = "0"
    sp2 = C_.gemm2_splits(N, K, T)
    os.environ["HSD_GEMM3"] = MASK
    sp3 = C_.gemm2_splits(N, K, T)
    os.environ["HSD_GEMM3"] = "0"
    ws = torch.empty(max(sp2, sp3) * N * K, device=dev)

    def run(i, dy=dy, x=x, sp=None, gws=gws, ws=ws):
        return C_.gemm2(dy, x, gws[i], 1, 1, 7, None, None, None, 0.0, 0, sp, ws, None)

    with_g3(False, lambda: run(0, sp=sp2))
    with_g3(True, lambda: run(1, sp=sp3))
    torch.cuda.synchronize()
    ref = dy[:, :256].float().t() @ x.float()
    rec = {"splits2": sp2, "splits3": sp3,
           "err2": ((gws[0][:256] - ref).abs().max() / ref.abs().max()).item(),
           "err3": ((gws[1][:256] - ref).abs().max() / ref.abs().max()).item()}
    out[name] = rec
    cases[name] = (2.0 * N * K * T, lambda run=run, sp2=sp2: run(0, sp=sp2), lambda run=run, sp3=sp3: run(1, sp=sp3))
    print("checked", name, rec, flush=True)

res = {k: {"g2": [], "g3": []} for k in cases}
for r in range(ROUNDS):
    for k, (fl, f2, f3) in cases.items():
        res[k]["g2"].append(fl / with_g3(False, lambda: timeit(f2)) / 1e12)
        res[k]["g3"].append(fl / with_g3(True, lambda: timeit(f3)) / 1e12)
tot2 = tot3 = 0.0
for k, (fl, _, _) in cases.items():
    g2 = sorted(res[k]["g2"])[len(res[k]["g2"]) // 2]
    g3 = sorted(res[k]["g3"])[len(res[k]["g3"]) // 2]
    out[k].update({"TF_g2": round(g2, 1), "TF_g3": round(g3, 1), "us_g2": round(fl / g2 / 1e6, 1),
                   "us_g3": round(fl / g3 / 1e6, 1)})
    tot2 += fl / g2 / 1e6
    tot3 += fl / g3 / 1e6
    print(k, out[k], flush=True)
out["_sum_us"] = {"g2": round(tot2, 1), "g3": round(tot3, 1)}
print("sum us", out["_sum_us"])
os.makedirs("gpurun_out", exist_ok=True)
json.dump(out, open("gpurun_out/gemm3_probe.json", "w"), indent=1)
