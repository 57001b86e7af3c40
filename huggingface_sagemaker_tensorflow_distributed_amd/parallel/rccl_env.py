"""RCCL defaults for one MI355X node (SURVEY.md §2.5 C.2, §5 'distributed communication backend').

The reference tunes its NCCL data plane only through commented-out MPI options (``/root/reference/launch.py:22``:
``--NCCL_DEBUG=INFO``). RCCL reads the same ``NCCL_*`` variables. They must be in the environment before the first
communicator is created (``torch.distributed`` with backend ``nccl`` and the native ``CommEngine`` both create one),
so :func:`apply` runs at the top of :func:`parallel.backend.init`. A variable the user already set is never
changed; ``HSD_RCCL_DEFAULTS=0`` turns the whole policy off.

Why these values (8 GPUs, every pair joined by one xGMI link, 7 links per GPU, ~153 GB/s each way):

* ``NCCL_MIN_NCHANNELS`` = 7 x 2. A channel is one ring; a ring leaves every GPU on ONE outgoing link, so a
  collective only spans all 7 links of a GPU when at least 7 rings run (the directed complete graph on 8 GPUs
  splits into exactly 7 link-disjoint Hamiltonian rings), and two channels per link keep each link busy while the
  other channel's chunk is in the reduce step.
* ``NCCL_MAX_NCHANNELS`` = 7 x 4. Every channel is one RCCL workgroup that holds a CU for the collective's duration,
  while the gradient all-reduces overlap the backward GEMMs (persistent, one 512-thread workgroup per CU). What a
  held CU costs those GEMMs was measured, not estimated (``tools/contention_ab.py``,
  ``profiles/contention_ab_r4.jsonl``): k whole CUs held for 400 us by a side-stream kernel (``cu_hog``, the RCCL
  stand-in) during one bert-base GEMM at T = 131072. With the dynamic tile queue (``gemm_common.h`` tq_*, default)
  a late workgroup takes fewer tiles, and k = 14 / 28 / 56 cost qkv_fwd +1.9 / +4.9 / +10.9 % (proportional CU loss:
  +5.4 / +10.8 / +21.6 %), while ffn1_fwd and ffn2_dgrad, whose epilogues are bound by the chip's store rate rather
  than by CUs, ran 3-7 % FASTER with CUs held. With the old static tile walk the same holds cost +71-78 % on qkv_fwd
  and +26-28 % on ffn2_dgrad. So the cap is set by link saturation (4 channels per link), not by CU pressure: 28 channels
  held through a bucket's all-reduce cost the overlapped GEMM at most ~5 %, and only for the bucket's ~0.1-0.2 ms.
* At N = 2 / 4 a GPU reaches 1 / 3 peers; the same floors and caps apply (RCCL lays several channels per link).

Bucket size (``--bucket_mb``, default 64 MiB, ``parallel/ddp.py``): bert-base's 418 MiB of fp32 gradients form 7
buckets in reverse layer order. Each all-reduce of 64 MiB at N = 8 moves 2 x 7/8 x 64 MiB per GPU, ~0.1-0.2 ms on the
links above: far above RCCL's latency floor (tens of us) and far below a layer's backward (~4 ms), so the first
bucket starts after ~1.5 layers of backward and every bucket but the last hides under the remaining backward.
"""
from __future__ import annotations

import logging
import os
from typing import Dict

logger = logging.getLogger(__name__)

XGMI_LINKS_PER_GPU = 7
DEFAULTS: Dict[str, str] = {
    "NCCL_MIN_NCHANNELS": str(2 * XGMI_LINKS_PER_GPU),
    "NCCL_MAX_NCHANNELS": str(4 * XGMI_LINKS_PER_GPU),
}


def apply(world_size: int) -> Dict[str, str]:
    """Set the defaults that are not already set (multi-rank worlds only). Returns what was set."""
    if world_size <= 1 or os.environ.get("HSD_RCCL_DEFAULTS", "1") == "0":
        return {}
    set_here = {}
    for k, v in DEFAULTS.items():
        if k not in os.environ:
            os.environ[k] = v
            set_here[k] = v
    if set_here:
        logger.info("RCCL defaults for xGMI: %s", " ".join(f"{k}={v}" for k, v in set_here.items()))
    return set_here


def effective() -> Dict[str, str]:
    """The NCCL_* / RCCL_* variables in force (reported in bench.py's JSON line)."""
    return {k: v for k, v in sorted(os.environ.items()) if k.startswith(("NCCL_", "RCCL_"))}
