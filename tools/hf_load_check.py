"""Load a checkpoint this framework saved with HF ``transformers`` and compare logits on one batch.

    python tools/hf_load_check.py <model_dir>

The reference's artefact contract (``scripts/train.py:182``): ``save_pretrained`` output that
``AutoModelForSequenceClassification.from_pretrained`` loads unchanged. The HF model runs in fp32 eager mode; this
framework's model is loaded from the same directory and runs its own forward (HIP kernels on a GPU, bf16 compute),
eval mode, same padded batch. Prints the max |logit difference| and the argmax agreement, exits non-zero on a
mismatch beyond bf16 tolerance.
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))

from huggingface_sagemaker_tensorflow_distributed_amd.models.hf_io import from_pretrained  # noqa: E402
from huggingface_sagemaker_tensorflow_distributed_amd.parallel import FlatParamStore  # noqa: E402


def main(path: str) -> int:
    from transformers import AutoModelForSequenceClassification

    dev = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    hf = AutoModelForSequenceClassification.from_pretrained(path).eval()
    ours = from_pretrained(path)
    cfg = ours.cfg
    g = torch.Generator().manual_seed(7)
    B, S = 16, 128
    ids = torch.randint(1000, cfg.vocab_size, (B, S), generator=g)
    am = torch.ones(B, S, dtype=torch.long)
    for b in range(B):  # variable real lengths, padded to S as in the reference (pad id 0)
        n = int(torch.randint(16, S + 1, (1,), generator=g))
        am[b, n:] = 0
        ids[b, n:] = cfg.pad_token_id
    with torch.no_grad():
        ref = hf(input_ids=ids, attention_mask=am).logits.float()
    ours = ours.to(dev).eval()
    compute = torch.bfloat16 if dev.type == "cuda" else torch.float32
    FlatParamStore(ours, dev, compute_dtype=compute)
    with torch.no_grad():
        got = ours(ids.to(dev), attention_mask=am.to(dev)).float().cpu()
    diff = (got - ref).abs().max().item()
    agree = (got.argmax(-1) == ref.argmax(-1)).float().mean().item()
    scale = ref.abs().max().item()
    tol = 0.05 * max(scale, 1.0) if compute == torch.bfloat16 else 1e-4
    ok = diff <= tol
    print(json.dumps({"model_dir": path, "architecture": type(hf).__name__, "device": str(dev),
                      "compute_dtype": str(compute).replace("torch.", ""), "batch": [B, S],
                      "max_abs_logit_diff": diff, "logit_scale": scale, "tol": tol,
                      "argmax_agreement": agree, "ok": ok}))
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
