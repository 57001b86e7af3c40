"""Speed-of-light table for the headline step's GEMMs (bert-base, B = 1024, S = 128: T = 131,072 tokens).

    rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES \
        --output-format csv -d gpurun_out/sol -o run -- python tools/gemm_sol.py run
    python tools/gemm_sol.py report gpurun_out/sol > profiles/gemm_sol_r2.json

`run` launches each of the layer's 12 GEMMs (the epilogues the step uses, random operands) REPS times in a fixed
order; `report` joins the per-dispatch counters: wall time, TFLOP/s, the effective clock (GRBM_GUI_ACTIVE / 8 XCDs
/ wall, MI355X_MICROARCH.md 'DVFS give-back') and the fraction of the MFMA peak AT THAT CLOCK
(256 CUs x 4 SIMDs x 1024 bf16 FLOP / cycle), next to the fraction of the 2.5 PFLOP/s nameplate.
Profiled passes run a few % slower than unprofiled ones (same note); compare rows, not runs."""
import collections
import csv
import glob
import json
import os
import sys

T = int(os.environ.get("SOL_T", "131072"))
H = int(os.environ.get("SOL_H", "768"))  # bert-large S=512 B=64: SOL_T=32768 SOL_H=1024
I = 4 * H
REPS = 6
# name: (layout, M, N, K, epi)  -- NT: C[M][N] = A[M][K] B[N][K]^T;  TT: dW[N][K] += dY[T][N]^T X[T][K]
GEMMS = [
    ("qkv_fwd_bias", "NT", T, 3 * H, H, 1), ("out_fwd_drop_res", "NT", T, H, H, 3),
    ("ffn1_fwd_gelu_d", "NT", T, I, H, 8), ("ffn2_fwd_drop_res", "NT", T, H, I, 3),
    ("ffn2_dgrad_mul_dbias", "NT", T, I, H, 9), ("ffn1_dgrad_res", "NT", T, H, I, 4),
    ("out_dgrad", "NT", T, H, H, 0), ("qkv_dgrad_res", "NT", T, H, 3 * H, 4),
    ("qkv_wgrad", "TT", 3 * H, H, T, 7), ("out_wgrad", "TT", H, H, T, 7),
    ("ffn1_wgrad", "TT", I, H, T, 7), ("ffn2_wgrad", "TT", H, I, T, 7),
]


def run():
    import torch

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from huggingface_sagemaker_tensorflow_distributed_amd.ops import hip

    C_ = hip._C
    dev = "cuda"
    rnd = lambda *s: (torch.rand(*s, device=dev) * 2 - 1).bfloat16()  # noqa: E731
    for name, lay, M, N, K, epi in GEMMS:
        if lay == "NT":
            a, b = rnd(M, K), rnd(N, K) * 0.05
            bias, aux = rnd(N), rnd(M, N)
            c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            c2 = torch.empty_like(c) if epi in (2, 8) else None
            db = torch.zeros(N, device=dev) if epi in (5, 9) else None
            fn = lambda: C_.gemm2(a, b, c, 0, 0, epi, bias if epi in (1, 2, 3, 8) else None,  # noqa: E731
                                  aux if epi in (3, 4, 5, 9) else None, c2, 0.1 if epi == 3 else 0.0, 7, 1, None, db)
        else:
            dy, x = rnd(K, M), rnd(K, N)  # tokens x out-features, tokens x in-features
            g = torch.zeros(M, N, device=dev)
            sp = C_.gemm2_splits(M, N, K)
            ws = torch.empty(sp * M * N, device=dev)
            fn = lambda: C_.gemm2(dy, x, g, 1, 1, 7, None, None, None, 0.0, 0, sp, ws, None)  # noqa: E731
        for _ in range(REPS):
            fn()
        torch.cuda.synchronize()
        print(name, flush=True)


def report(d):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    per = collections.defaultdict(dict)
    for r in rows:
        if "gemm2_kernel" not in r["Kernel_Name"]:
            continue
        k = int(r["Dispatch_Id"])
        per[k][r["Counter_Name"]] = float(r["Counter_Value"])
        per[k]["dur_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    disp = [per[k] for k in sorted(per)]
    assert len(disp) == REPS * len(GEMMS), f"{len(disp)} gemm2 dispatches, expected {REPS * len(GEMMS)}"
    out = {}
    for i, (name, lay, M, N, K, epi) in enumerate(GEMMS):
        ds = disp[i * REPS + 1:(i + 1) * REPS]  # first call of each shape is a warm-up
        dur = sorted(x["dur_ns"] for x in ds)[len(ds) // 2] * 1e-9
        f = sorted(x["GRBM_GUI_ACTIVE"] / 8 / (x["dur_ns"] * 1e-9) for x in ds)[len(ds) // 2]
        tf = 2.0 * M * N * K / dur / 1e12
        peak_at_f = 256 * 4 * 1024 * f / 1e12
        out[name] = {"M": M, "N": N, "K": K, "epi": epi, "us": round(dur * 1e6, 1), "TFLOPs": round(tf, 1),
                     "eff_clock_GHz": round(f / 1e9, 3), "pct_of_peak_at_clock": round(100 * tf / peak_at_f, 1),
                     "pct_of_2.5PF": round(100 * tf / 2500, 1)}
    tot_fl = sum(2.0 * M * N * K for _, _, M, N, K, _ in GEMMS)
    tot_us = sum(v["us"] for v in out.values())
    out["_layer"] = {"us": round(tot_us, 1), "TFLOPs": round(tot_fl / (tot_us * 1e-6) / 1e12, 1)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run()
    else:
        report(sys.argv[2])
