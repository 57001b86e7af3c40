"""This framework's GEMMs vs hipBLASLt (torch.addmm / torch.mm) on the headline layer's shapes, one process.

    python tools/vs_hipblaslt.py [T [H]]  (default T = 131072 tokens = bert-base B = 1024, S = 128; H = 768;
                                          bert-large B = 8 S = 512: 4096 1024)

For each bert-base projection (QKV, attention output, FFN1, FFN2) and each of its three GEMMs:
  forward  y = x Wᵀ + b        ours: gemm2 NT, bias epilogue      library: torch.addmm(b, x, Wᵀ)
  dgrad    dx = dy W           ours: gemm2 NT on the stored Wᵀ    library: torch.mm(dy, W)
  wgrad    dW += dyᵀ x (fp32)  ours: gemm2 TT split-K + reduce    library: main_grad += torch.mm(dyᵀ, x) (bf16 out)
  wgrad_f32                    same                                library: torch.addmm(main_grad, dyᵀ, x, out_dtype=fp32)
Random operands, HIP-event timing, interleaved rounds (ours / library alternate) so both see the same clocks.
Prints one JSON object (TFLOP/s per GEMM and the layer totals); also writes gpurun_out/vs_hipblaslt.json.
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from huggingface_sagemaker_tensorflow_distributed_amd.ops import hip  # noqa: E402


def timed(fn, iters=10):
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(iters):
        fn()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / iters * 1e-3


def _addmm_f32(c, a, b):
    """c += a @ b with bf16 inputs and the fp32 output / accumulation done by hipBLASLt (aten::addmm.dtype)."""
    try:
        torch.addmm(c, a, b, out_dtype=torch.float32, out=c)
    except (RuntimeError, TypeError):
        c.copy_(torch.addmm(c, a, b, out_dtype=torch.float32))


def main():
    T = int(sys.argv[1]) if len(sys.argv) > 1 else 131072
    H = int(sys.argv[2]) if len(sys.argv) > 2 else 768
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    out = {"tokens": T, "hidden": H}
    tot = {"ours_s": 0.0, "lib_s": 0.0, "flop": 0.0}
    for name, (N, K) in {"qkv": (3 * H, H), "attn_out": (H, H), "ffn1": (4 * H, H),
                         "ffn2": (H, 4 * H)}.items():
        x = torch.randn(T, K, device=dev).bfloat16()
        w = torch.randn(N, K, device=dev).bfloat16() * 0.05
        wt = w.t().contiguous()
        b = torch.randn(N, device=dev).bfloat16()
        dy = torch.randn(T, N, device=dev).bfloat16()
        gw = torch.zeros(N, K, device=dev)
        w.main_grad = gw
        g = hip._Grad(w)
        fl = 2.0 * T * N * K
        cases = {
            "fwd": (lambda: hip.gemm_fwd(x, w, hip.EPI_BIAS, bias=b), lambda: torch.addmm(b, x, w.t())),
            "dgrad": (lambda: hip._C.gemm2(dy, wt, torch.empty(T, K, device=dev, dtype=torch.bfloat16), 0, 0,
                                           hip.EPI_STORE, None, None, None, 0.0, 0, 0, None, None),
                      lambda: torch.mm(dy, w)),
            "wgrad": (lambda: hip.gemm_wgrad_(g, dy, x), lambda: gw.add_(torch.mm(dy.t(), x))),
            # the like-for-like library comparator: fp32 output accumulated into main_grad by the GEMM itself
            "wgrad_f32": (lambda: hip.gemm_wgrad_(g, dy, x), lambda: _addmm_f32(gw, dy.t(), x)),
        }
        r = {}
        for case, (ours, lib) in cases.items():
            for f in (ours, lib):  # warm-up (kernel selection, workspaces)
                f()
                f()
            torch.cuda.synchronize()
            t_o, t_l = [], []
            for _ in range(3):
                t_o.append(timed(ours))
                t_l.append(timed(lib))
            to, tl = min(t_o), min(t_l)
            r[case] = {"ours_TFLOPs": round(fl / to / 1e12, 1), "hipblaslt_TFLOPs": round(fl / tl / 1e12, 1),
                       "ours_us": round(to * 1e6, 1), "hipblaslt_us": round(tl * 1e6, 1), "speedup": round(tl / to, 3)}
            if case != "wgrad":  # layer totals use the fp32-output comparator
                tot["ours_s"] += to
                tot["lib_s"] += tl
                tot["flop"] += fl
        out[name] = r
        print(name, json.dumps(r), flush=True)
        del w.main_grad
    out["layer"] = {"ours_TFLOPs": round(tot["flop"] / tot["ours_s"] / 1e12, 1),
                    "hipblaslt_TFLOPs": round(tot["flop"] / tot["lib_s"] / 1e12, 1),
                    "speedup": round(tot["lib_s"] / tot["ours_s"], 3)}
    print(json.dumps(out), flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    json.dump(out, open("gpurun_out/vs_hipblaslt.json", "w"), indent=1)


if __name__ == "__main__":
    main()
