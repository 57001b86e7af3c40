"""TT weight-gradient GEMM schedule / split probe on the headline shapes (interleaved rounds, one process).

    PROBE_SYNC=0,4,5,6,7 PROBE_SPLITS=auto,4,7,14 python tools/tt_probe.py [T]   -> gpurun_out/tt_probe.json

For each bert-base weight (dW[N][K] += dy[T][N]ᵀ x[T][K]) every (HSD_G2_SYNC schedule, K-split count) pair is
timed with HIP events and checked against the first pair's result (fp32, same inputs)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from huggingface_sagemaker_tensorflow_distributed_amd.ops import hip  # noqa: E402

C_ = hip._C
T = int(sys.argv[1]) if len(sys.argv) > 1 else 131072
SYNCS = [int(v) for v in os.environ.get("PROBE_SYNC", "0,4,7").split(",")]
SPLITS = os.environ.get("PROBE_SPLITS", "auto").split(",")
SHAPES = {"qkv": (2304, 768), "attn_out": (768, 768), "ffn1": (3072, 768), "ffn2": (768, 3072)}


def timeit(fn, iters=8):
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(iters):
        fn()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / iters * 1e-3


def main():
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    out = {"tokens": T}
    for name, (N, K) in SHAPES.items():
        dy = torch.randn(T, N, device=dev).bfloat16()
        x = torch.randn(T, K, device=dev).bfloat16()
        fl = 2.0 * T * N * K
        auto = C_.gemm2_splits(N, K, T)
        ws = torch.empty(64 * N * K, device=dev)
        variants = []
        for sync in SYNCS:
            for sp in SPLITS:
                variants.append((sync, auto if sp == "auto" else int(sp)))
        ref = None
        times = {v: [] for v in variants}
        for rnd in range(3):
            for v in variants:
                os.environ["HSD_G2_SYNC"] = str(v[0])
                hip._C.refresh_env()  # launch knobs are cached (common.h HSD_KNOB)
                g = torch.zeros(N, K, device=dev)

                def run():
                    C_.gemm2(dy, x, g, 1, 1, 7, None, None, None, 0.0, 0, v[1], ws, None)
                run()
                torch.cuda.synchronize()
                if rnd == 0:
                    if ref is None:
                        ref = g.clone()
                    else:
                        err = float((g - ref).abs().max() / ref.abs().max())
                        assert err < 1e-4, (name, v, err)
                times[v].append(timeit(run))
        os.environ.pop("HSD_G2_SYNC", None)
        hip._C.refresh_env()  # launch knobs are cached (common.h HSD_KNOB)
        r = {}
        for v, ts in times.items():
            t = min(ts)
            r[f"sync{v[0]}_s{v[1]}"] = {"us": round(t * 1e6, 1), "TFLOPs": round(fl / t / 1e12, 1)}
        r["auto_splits"] = auto
        out[name] = r
        best = min((k for k in r if k != "auto_splits"), key=lambda k: r[k]["us"])
        print(name, "auto", auto, "best", best, r[best], json.dumps(r), flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    json.dump(out, open("gpurun_out/tt_probe.json", "w"), indent=1)


if __name__ == "__main__":
    main()
