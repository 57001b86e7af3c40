"""Cost of a stream fork (hipEventRecord on the producer stream + hipStreamWaitEvent on the consumer) on the PRODUCER's
critical path: a chain of N short dependent-order kernels on the main stream, with and without a fork after each.

    python tools/fork_cost.py [N] [usec]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from huggingface_sagemaker_tensorflow_distributed_amd.ops import hip  # noqa: E402

C = hip._C
N = int(sys.argv[1]) if len(sys.argv) > 1 else 400
us = float(sys.argv[2]) if len(sys.argv) > 2 else 3.0
dev = torch.device("cuda", 0)
main = torch.cuda.Stream(device=dev)
side = torch.cuda.Stream(device=dev)


def run(mode):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.cuda.stream(main):
        for i in range(N):
            C.cu_hog(1, us)
            if mode == "fork":  # side waits for main (event recorded on main)
                C.stream_wait(side.cuda_stream, main.cuda_stream)
            elif mode == "fork+work":  # ... and runs a kernel of its own
                C.stream_wait(side.cuda_stream, main.cuda_stream)
                with torch.cuda.stream(side):
                    C.cu_hog(1, us)
            elif mode == "join":  # main waits for side (event recorded on side)
                C.stream_wait(main.cuda_stream, side.cuda_stream)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / N * 1e6


for mode in ("plain", "fork", "fork+work", "join", "plain", "fork"):
    run(mode)
    r = sorted(run(mode) for _ in range(5))
    print(f"{mode:10s} {r[2]:7.2f} us per kernel (N={N}, kernel {us} us)", flush=True)
