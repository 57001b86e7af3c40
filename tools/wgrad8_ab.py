"""fp8 vs bf16 weight gradient (dW[M][N] += dyᵀ·x over T tokens): gemm2.hip gemm8tt_kernel (+ slab reduce) on the
producers' fp8 copies vs the bf16 TT kernel (gemm2_kernel<1,1,7>) on the bf16 tensors. One JSON line per shape with
the median time of each and the TFLOP/s.  python tools/wgrad8_ab.py [iters]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from huggingface_sagemaker_tensorflow_distributed_amd.ops import hip  # noqa: E402

dev = "cuda"
iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
shapes = [  # (name, M = out features, N = in features, T tokens)
    ("rl_qkv", 3072, 1024, 32768), ("rl_out", 1024, 1024, 32768), ("rl_ffn1", 4096, 1024, 32768),
    ("rl_ffn2", 1024, 4096, 32768),
    ("bb_qkv", 2304, 768, 131072), ("bb_out", 768, 768, 131072), ("bb_ffn1", 3072, 768, 131072),
    ("bb_ffn2", 768, 3072, 131072),
]


def timeit(fn):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


hip.set_fp8(True)
for name, M, N, T in shapes:
    torch.manual_seed(0)
    dy = (torch.randn(T, M, device=dev) * 0.01).bfloat16()
    x = torch.randn(T, N, device=dev).bfloat16()
    qd, sd = hip.quant_fp8(dy, 0)
    qx, sx = hip.quant_fp8(x, 0)
    buf = torch.zeros(M, N, device=dev)

    class G:
        pass

    g = G()
    g.buf = buf
    t16 = timeit(lambda: hip.gemm_wgrad_(g, dy, x))
    t8 = timeit(lambda: hip._wgrad8(buf, (qd, sd), (qx, sx), M, N, T))
    fl = 2.0 * M * N * T
    print(json.dumps({"shape": name, "M": M, "N": N, "T": T, "bf16_us": round(t16, 1), "fp8_us": round(t8, 1),
                      "speedup": round(t16 / t8, 3), "bf16_tflops": round(fl / t16 / 1e6, 1),
                      "fp8_tflops": round(fl / t8 / 1e6, 1),
                      "splits8": hip._C.gemm8_wgrad_ws_numel(M, N, T, 0) // (M * N)}), flush=True)
hip.set_fp8(False)
