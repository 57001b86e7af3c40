"""Serving-style benchmark: forward-only (eval mode, dropout off) sequence-classification throughput and latency on
one GPU through the HIP kernels, eager or replayed from a captured HIP graph (the launch-bound small batches of
online serving).

    python tools/bench_infer.py [--model bert-base-uncased] [--seq_len 128] [--batches 1,8,64,1024] [--graph]

One JSON line per batch size: sequences/sec and ms per forward (median of 5 rounds). Synthetic full-length
token ids, random-init weights (offline box)."""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from huggingface_sagemaker_tensorflow_distributed_amd.models import build_model, resolve_config  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="bert-base-uncased")
    ap.add_argument("--seq_len", type=int, default=128)
    ap.add_argument("--batches", default="1,8,64,1024")
    ap.add_argument("--graph", action="store_true")
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    cfg = resolve_config(a.model)
    model = build_model(cfg, seed=0).to(dev).bfloat16().eval()
    for B in [int(x) for x in a.batches.split(",")]:
        ids = torch.randint(1000, cfg.vocab_size, (B, a.seq_len), device=dev)
        am = torch.ones(B, a.seq_len, dtype=torch.long, device=dev)

        def fwd():
            with torch.no_grad():
                return model(ids, attention_mask=am)

        for _ in range(3):
            fwd()
        torch.cuda.synchronize()
        run = fwd
        if a.graph:
            g = torch.cuda.CUDAGraph()
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                fwd()
                torch.cuda.synchronize()
                with torch.cuda.graph(g):
                    fwd()
            torch.cuda.current_stream().wait_stream(s)
            run = g.replay
        times = []
        for _ in range(5):
            st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            st.record()
            for _ in range(a.iters):
                run()
            en.record()
            torch.cuda.synchronize()
            times.append(st.elapsed_time(en) / a.iters)
        ms = statistics.median(times)
        print(json.dumps({"mode": "inference", "model": a.model, "seq_len": a.seq_len, "batch": B,
                          "graph": a.graph, "ms_per_forward": round(ms, 4),
                          "sequences_per_sec": round(B / (ms * 1e-3), 1), "dtype": "bf16",
                          "data": "synthetic, random-init weights"}), flush=True)


if __name__ == "__main__":
    main()
