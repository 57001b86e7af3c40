"""Convergence check on one GPU: bert-base sequence classification on the learnable synthetic task (the label is
carried by a marker token at a random position of a variable-length, padded sequence), trained with the HIP kernels
and, from the same initial weights and batches, with the plain torch reference ops (HSD_OPS=torch). Prints one
JSON line per path: the loss curve (mean over 25-step windows) and held-out loss / accuracy.

    python tools/convergence.py            # runs both paths as subprocesses
    python tools/convergence.py --path hip  # one path in this process"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _model_dir(layers: int) -> str:
    """bert-base width and vocab with ``layers`` encoder layers, as an HF config.json directory."""
    import tempfile

    d = tempfile.mkdtemp(prefix="hsd-conv-")
    cfg = {"model_type": "bert", "architectures": ["BertForSequenceClassification"], "vocab_size": 30522,
           "hidden_size": 768, "num_hidden_layers": layers, "num_attention_heads": 12, "intermediate_size": 3072,
           "hidden_act": "gelu", "hidden_dropout_prob": 0.1, "attention_probs_dropout_prob": 0.1,
           "max_position_embeddings": 512, "type_vocab_size": 2, "initializer_range": 0.02, "layer_norm_eps": 1e-12,
           "pad_token_id": 0, "num_labels": 2}
    with open(os.path.join(d, "config.json"), "w") as f:
        json.dump(cfg, f)
    return d


def one(path: str, steps: int, bs: int, seq: int, lr: float, layers: int = 12) -> dict:
    sys.path.insert(0, ROOT)
    import torch

    from huggingface_sagemaker_tensorflow_distributed_amd import data as hdata
    from huggingface_sagemaker_tensorflow_distributed_amd.data.loader import BatchLoader
    from huggingface_sagemaker_tensorflow_distributed_amd.parallel import ShardSampler
    from huggingface_sagemaker_tensorflow_distributed_amd.train.runner import build
    from huggingface_sagemaker_tensorflow_distributed_amd.utils.args import build_parser

    args, _ = build_parser("train").parse_known_args(
        ["--model_name_or_path", "bert-base-uncased" if layers == 12 else _model_dir(layers),
         "--train_batch_size", str(bs), "--learning_rate", str(lr),
         "--dtype", "bf16", "--log_every", "0", "--seed", "7"])
    parts = build(args, "train")
    tr, dev = parts["trainer"], parts["device"]
    ds = hdata.synthetic_classification(bs * steps, seq, 30522, seed=1)
    test = hdata.synthetic_classification(1024, seq, 30522, seed=2)
    curve, window = [], []
    for i in range(steps):
        sl = slice(i * bs, (i + 1) * bs)
        mb = {"input_ids": torch.from_numpy(ds.input_ids[sl]).long().to(dev),
              "attention_mask": torch.from_numpy(ds.attention_mask[sl]).long().to(dev),
              "labels": torch.from_numpy(ds.labels[sl]).long().to(dev)}
        window.append(float(tr.train_step([mb]).detach()))
        if len(window) == 25:
            curve.append(round(sum(window) / 25, 4))
            window = []
    loader = BatchLoader(test, ShardSampler(len(test), 0, 1, shuffle=False, drop_last=False, batch_size=64), dev)
    ev = tr.evaluate(loader)
    return {"path": path, "layers": layers, "steps": steps, "batch": bs, "seq_len": seq, "lr": lr, "loss_curve_25": curve,
            "eval_loss": round(ev["loss"], 4), "eval_accuracy": round(ev["sparse_categorical_accuracy"], 4)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--path", choices=["hip", "torch"], default=None)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--seq_len", type=int, default=128)
    ap.add_argument("--lr", type=float, default=3e-5)
    ap.add_argument("--layers", type=int, default=12, help="encoder layers (bert-base width)")
    a = ap.parse_args()
    if a.path:
        print(json.dumps(one(a.path, a.steps, a.batch, a.seq_len, a.lr, a.layers)), flush=True)
        return
    for path in ("hip", "torch"):
        env = dict(os.environ, HSD_OPS="torch" if path == "torch" else "")
        cmd = [sys.executable, os.path.abspath(__file__), "--path", path, "--steps", str(a.steps), "--batch",
               str(a.batch), "--seq_len", str(a.seq_len), "--lr", str(a.lr), "--layers", str(a.layers)]
        out = subprocess.run(cmd, env=env, capture_output=True, text=True)
        line = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
        print(line[-1] if line else json.dumps({"path": path, "error": out.stderr[-2000:]}), flush=True)


if __name__ == "__main__":
    main()
