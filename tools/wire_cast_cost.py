"""Cost of the bf16 gradient wire format on one GPU: the native engine's bucket path with
compression none vs bf16 (fp32 -> bf16 cast, all-reduce, bf16 -> fp32 cast, all on the comm stream) over the flat
gradient buffer of bert-base (109.5M) and bert-large (335.1M) at the default 64 MiB buckets, world-of-one RCCL
communicator. Prints one JSON line per (model, mode): ms per step of bucket traffic, and the difference = what the
two casts add per step on this rank.

    python tools/wire_cast_cost.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from huggingface_sagemaker_tensorflow_distributed_amd.ops._ext import load  # noqa: E402

C = load()
dev = torch.device("cuda", 0)
BUCKET = 64 << 20
for name, numel in (("bert-base-uncased", 109_483_778), ("bert-large-uncased", 335_143_938)):
    numel = (numel + 63) // 64 * 64  # FlatParamStore segments are 64-element aligned
    flat = torch.randn(numel, device=dev)
    per = BUCKET // 4
    starts = list(range(0, numel, per))
    ends = [min(s + per, numel) for s in starts]
    res = {}
    for mode in (0, 1):
        eng = C.CommEngine(0, 1, C.CommEngine.unique_id(), 0, True)
        eng.set_buckets(flat, starts, ends, [1] * len(starts), list(range(len(starts))))
        eng.set_compression(mode)
        st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        times = []
        for it in range(12):
            torch.cuda.synchronize()
            st.record()
            eng.begin_step()
            for i in range(len(starts)):
                eng.mark_ready(i)
            eng.finish()
            en.record()
            torch.cuda.synchronize()
            if it >= 2:
                times.append(st.elapsed_time(en))
        eng.close()
        times.sort()
        res[mode] = times[len(times) // 2]
        print(json.dumps({"model": name, "grad_numel": numel, "buckets": len(starts),
                          "wire": "bf16" if mode else "fp32", "ms_per_step_median": round(res[mode], 4)}), flush=True)
    print(json.dumps({"model": name, "cast_ms_per_step": round(res[1] - res[0], 4),
                      "note": "world-of-one: the all-reduce itself is a local pass; the difference is the two casts"}),
          flush=True)
    del flat
    torch.cuda.empty_cache()
