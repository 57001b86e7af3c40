"""The MLM head's dgrad dy = dlogits [n x Vp] . Wemb [Vp x H] (NT reading the table as its k-strided B, K = Vp ~ 50k):
time per tile / split choice.  python tools/mlm_dgrad_probe.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from huggingface_sagemaker_tensorflow_distributed_amd.ops import hip  # noqa: E402

C_ = hip._C
dev = "cuda"
M, N, K = 4928, 1024, 50432
a = (torch.randn(M, K, device=dev) * 0.01).bfloat16()
w = (torch.randn(K, N, device=dev) * 0.05).bfloat16()
c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
ws = torch.empty(8 * M * N, device=dev)


def run(env, splits):
    for k, v in env.items():
        os.environ[k] = v
    C_.refresh_env()
    f = lambda: C_.gemm2(a, w, c, 0, 1, 0, None, None, None, 0.0, 0, splits, ws, None)  # noqa: E731
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    ts = []
    for _ in range(10):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        f()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) * 1e3)
    for k in env:
        del os.environ[k]
    C_.refresh_env()
    ts.sort()
    return ts[5]


ref = None
for name, env, sp in [("default", {}, 0), ("small_sk2", {"HSD_G2_SMALL": "1"}, 2), ("small_sk4", {"HSD_G2_SMALL": "1"}, 4),
                      ("small_s3", {"HSD_G2_SMALL": "1", "HSD_G2S_STAGES": "3"}, 1),
                      ("big_sk3", {"HSD_G2_SMALL": "0"}, 3), ("big_sk1", {"HSD_G2_SMALL": "0"}, 1),
                      ("big_sk6", {"HSD_G2_SMALL": "0"}, 6)]:
    t = run(env, sp)
    out = c.float().clone()
    if ref is None:
        ref = out
    err = float((out - ref).abs().max())
    print(json.dumps({"case": name, "us": round(t, 1), "tflops": round(2 * M * N * K / t / 1e6, 1), "maxdiff": err}),
          flush=True)
