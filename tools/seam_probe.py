"""Where a persistent NT GEMM round goes: per workgroup and tile, shader-clock stamps after the main loop (t0), after
the epilogue issued its last store (t1) and after the seam wait + barrier (t2) (gemm2_set_diag, wave 0).
    python tools/seam_probe.py -> one JSON line per GEMM: mean cycles of main loop / epilogue / seam, clock (GHz)"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from huggingface_sagemaker_tensorflow_distributed_amd.ops import hip  # noqa: E402

C_ = hip._C
dev = "cuda"
T = 131072
rnd = lambda *s: (torch.rand(*s, device=dev) * 2 - 1).bfloat16()  # noqa: E731
diag = torch.zeros(256 * 64 * 4, dtype=torch.int64, device=dev)
for (N, K, epi) in [(3072, 64, 0), (3072, 768, 0), (3072, 768, 8), (3072, 768, 9), (2304, 768, 1), (768, 768, 3),
                    (768, 768, 0), (768, 3072, 4), (768, 3072, 3)]:
    a, b, bias, aux = rnd(T, K), rnd(N, K) * 0.05, rnd(N), rnd(T, N)
    c, c2 = torch.empty(T, N, device=dev, dtype=torch.bfloat16), torch.empty(T, N, device=dev, dtype=torch.bfloat16)
    db = torch.zeros(N, device=dev) if epi in (5, 9) else None

    def fn():
        C_.gemm2(a, b, c, 0, 0, epi, bias if epi in (1, 2, 3, 8) else None, aux if epi in (3, 4, 5, 9) else None,
                 c2 if epi in (2, 8) else None, 0.1 if epi == 3 else 0.0, 7, 1, None, db)

    for _ in range(3):
        fn()
    diag.zero_()
    C_.gemm2_set_diag(diag)
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    fn()
    en.record()
    torch.cuda.synchronize()
    C_.gemm2_set_diag(None)
    d = diag.view(256, 64, 4).cpu().double()
    valid = d[:, :, 3] > 0
    t0, t1, t2, rt = d[..., 0], d[..., 1], d[..., 2], d[..., 3]
    epi_c = (t1 - t0)[valid]
    seam_c = (t2 - t1)[valid]
    # main loop of tile i (i >= 1) = t0[i] - t2[i-1]
    v2 = valid[:, 1:] & valid[:, :-1]
    main_c = (t0[:, 1:] - t2[:, :-1])[v2]
    clk = ((t2[:, 1:] - t2[:, :-1]) / ((rt[:, 1:] - rt[:, :-1]) * 10.0))[v2]  # cycles per ns = GHz
    print(json.dumps({"N": N, "K": K, "epi": epi, "us": round(st.elapsed_time(en) * 1e3, 1),
                      "tiles_per_wg": int(valid.sum(1).float().mean()),
                      "main_cyc": round(float(main_c.mean()), 0) if main_c.numel() else None,
                      "epi_cyc": round(float(epi_c.mean()), 0), "seam_cyc": round(float(seam_c.mean()), 0),
                      "epi_cyc_p90": round(float(epi_c.quantile(0.9)), 0),
                      "clock_ghz": round(float(clk.median()), 3) if clk.numel() else None}), flush=True)
