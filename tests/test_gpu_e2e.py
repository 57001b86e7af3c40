"""End-to-end GPU checks: whole-model HIP path vs torch-reference path, and a short training run."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu

from huggingface_sagemaker_tensorflow_distributed_amd import ops  # noqa: E402
from huggingface_sagemaker_tensorflow_distributed_amd.models import build_model, resolve_config  # noqa: E402


def _run(model, ids, am, labels, force_torch):
    old = ops._FORCE_TORCH
    ops._FORCE_TORCH = force_torch
    try:
        model.zero_grad(set_to_none=True)
        model.rng.new_step(5)
        loss, logits = model(ids, attention_mask=am, labels=labels)
        loss.backward()
        return loss.detach().float(), logits.detach().float(), {n: p.grad.float().clone() for n, p in model.named_parameters()}
    finally:
        ops._FORCE_TORCH = old


@pytest.mark.parametrize("name", ["hsd-tiny-bert", "hsd-tiny-roberta", "hsd-tiny-distilbert"])
def test_model_hip_vs_reference(gpu, name):
    cfg = resolve_config(name).replace(hidden_size=128, num_attention_heads=2, intermediate_size=256)
    m = build_model(cfg, seed=0).to(gpu).bfloat16()
    torch.manual_seed(0)
    B, S = 4, 64
    ids = torch.randint(5, cfg.vocab_size, (B, S), device=gpu)
    am = torch.ones(B, S, dtype=torch.long, device=gpu)
    am[1, 40:] = 0
    labels = torch.randint(0, 2, (B,), device=gpu)
    l1, g1_logits, g1 = _run(m, ids, am, labels, False)
    l2, g2_logits, g2 = _run(m, ids, am, labels, True)
    assert torch.allclose(l1, l2, atol=2e-2, rtol=2e-2), (l1, l2)
    assert torch.allclose(g1_logits, g2_logits, atol=5e-2, rtol=5e-2)
    for n in g1:
        a, b = g1[n], g2[n]
        rel = (a - b).norm() / (b.norm() + 1e-6)
        assert rel < 5e-2, f"{n}: rel grad err {rel:.3g}"


def test_bert_base_train_steps_loss_decreases(gpu):
    from huggingface_sagemaker_tensorflow_distributed_amd import data as hdata
    from huggingface_sagemaker_tensorflow_distributed_amd.train.runner import build
    from huggingface_sagemaker_tensorflow_distributed_amd.utils.args import build_parser

    args, _ = build_parser("train").parse_known_args(
        ["--model_name_or_path", "bert-base-uncased", "--train_batch_size", "32", "--learning_rate", "5e-5",
         "--dtype", "bf16", "--log_every", "0", "--hip_graph", "false"])
    parts = build(args, "train")
    tr = parts["trainer"]
    ds = hdata.synthetic_classification(32 * 4, 128, 30522, seed=0)
    batches = []
    for i in range(4):
        sl = slice(32 * i, 32 * (i + 1))
        batches.append({k: torch.from_numpy(v[sl]).long().to(gpu) for k, v in
                        (("input_ids", ds.input_ids), ("attention_mask", ds.attention_mask), ("labels", ds.labels))})
    losses = []
    for step in range(40):
        losses.append(float(tr.train_step([batches[step % 4]])))
    assert all(l == l for l in losses), "NaN loss"
    assert sum(losses[-8:]) / 8 < sum(losses[:8]) / 8, losses


def test_store_transposed_weights_track_optimizer(gpu):
    """FlatParamStore keeps bf16 Wᵀ copies for the dgrad GEMMs in sync with the weights after each step."""
    from huggingface_sagemaker_tensorflow_distributed_amd.optim import FusedAdam
    from huggingface_sagemaker_tensorflow_distributed_amd.parallel import FlatParamStore

    cfg = resolve_config("hsd-tiny-bert").replace(hidden_size=256, num_attention_heads=4, intermediate_size=512)
    m = build_model(cfg, seed=0).to(gpu)
    store = FlatParamStore(m, gpu, compute_dtype=torch.bfloat16)
    opt = FusedAdam(store, lr=1e-3)
    tracked = [(n, p) for n, p in m.named_parameters() if hasattr(p, "_hsd_wt")]
    assert len(tracked) == 4 * cfg.num_hidden_layers
    ids = torch.randint(5, cfg.vocab_size, (2, 128), device=gpu)
    labels = torch.randint(0, 2, (2,), device=gpu)
    for _ in range(2):
        store.zero_grad()
        m.rng.new_step(0)
        loss, _ = m(ids, attention_mask=torch.ones_like(ids), labels=labels)
        loss.backward()
        opt.step()
        torch.cuda.synchronize()
        for n, p in tracked:
            assert torch.equal(p._hsd_wt, p.detach().t()), n


@pytest.mark.parametrize("model,seq,bs", [("bert-base-uncased", 128, 32), ("bert-large-uncased-whole-word-masking", 512, 8)])
def test_train_script_on_gpu_writes_reference_artifacts(gpu, tmp_path, model, seq, bs):
    """scripts/train.py end to end on the GPU (the reference's job: fit -> evaluate -> save_pretrained),
    including the reference's own bert-large-wwm S=512 configuration (launch.py:14-17)."""
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, SM_OUTPUT_DATA_DIR=str(tmp_path / "data"), SM_MODEL_DIR=str(tmp_path / "model"),
               SM_NUM_GPUS="1", SM_FRAMEWORK_PARAMS="{}")
    cmd = [sys.executable, os.path.join(root, "scripts", "train.py"), "--epochs", "1", "--train_batch_size", str(bs),
           "--eval_batch_size", "4", "--model_name_or_path", model, "--max_seq_length", str(seq),
           "--num_train_examples", str(bs * 4), "--num_eval_examples", "16", "--log_every", "1"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    train = (tmp_path / "data" / "train_results.txt").read_text()
    assert train.startswith("loss = [") and "sparse_categorical_accuracy = [" in train and "train_runtime = {" in train
    ev = (tmp_path / "data" / "eval_results.txt").read_text().splitlines()
    assert ev[0].startswith("loss = ") and ev[1].startswith("sparse_categorical_accuracy = ")
    cfg = json.loads((tmp_path / "model" / "config.json").read_text())
    assert cfg["architectures"] == ["BertForSequenceClassification"]
    assert (tmp_path / "model" / "model.safetensors").exists()


@pytest.mark.parametrize("accum", [1, 2])
def test_optimizer_overlapped_with_backward_uses_final_gradients(gpu, monkeypatch, accum):
    """Adam slices stepped under backward (LocalOverlap, the default on one GPU): after each step the master
    weights, moments and bf16 copies equal ONE full Adam pass applied afterwards to the final gradients of that step
    (bit for bit) -- a slice stepped before its last gradient landed, or with the wrong coefficients, would differ.
    Run-to-run comparison is not bitwise (fp32 atomics in the backward), hence this per-step replay."""
    from huggingface_sagemaker_tensorflow_distributed_amd import data as hdata
    from huggingface_sagemaker_tensorflow_distributed_amd.ops import hip
    from huggingface_sagemaker_tensorflow_distributed_amd.train.runner import build
    from huggingface_sagemaker_tensorflow_distributed_amd.utils.args import build_parser

    ds = hdata.synthetic_classification(8 * 4, 128, 30522, seed=0)
    batches = [{k: torch.from_numpy(v[8 * i:8 * (i + 1)]).long().to(gpu) for k, v in
                (("input_ids", ds.input_ids), ("attention_mask", ds.attention_mask), ("labels", ds.labels))}
               for i in range(4)]
    monkeypatch.setenv("HSD_OPT_OVERLAP", "1")
    monkeypatch.setenv("HSD_OPT_BUCKET_MB", "4")  # many slices
    monkeypatch.setenv("HSD_WT", "1")  # keep the Wᵀ copies at this small step (their per-slice refresh is checked)
    args, _ = build_parser("train").parse_known_args(
        ["--model_name_or_path", "bert-base-uncased", "--train_batch_size", "8", "--learning_rate", "1e-4",
         "--dtype", "bf16", "--log_every", "0", "--hip_graph", "false", "--seed", "3"])
    parts = build(args, "train")
    tr, st, opt = parts["trainer"], parts["store"], parts["optimizer"]
    tr.zero_grad_in_optimizer = False  # the replay below reads the step's final gradients after the step
    assert tr._opt_overlap is not None and len(opt._ranges) > 10
    for step in range(3):
        p0, m0, v0 = st.master.clone(), opt.exp_avg.clone(), opt.exp_avg_sq.clone()
        tr.train_step([batches[(step * accum + j) % 4] for j in range(accum)])
        torch.cuda.synchronize()
        s, eps = opt._coeffs()
        out = torch.empty_like(st.compute)
        hip.adam_step(p0, m0, v0, st.grad, out, None, s, eps, opt.beta1, opt.beta2, 1.0 / accum, 0.0)
        torch.cuda.synchronize()
        assert torch.equal(p0, st.master) and torch.equal(m0, opt.exp_avg) and torch.equal(v0, opt.exp_avg_sq)
        assert torch.equal(out, st.compute)
        # each slice's Wᵀ copies are refreshed right after its update
        tracked = [p for p in st.params if hasattr(p, "_hsd_wt")]
        assert len(tracked) == 48
        for p in tracked:
            assert torch.equal(p._hsd_wt, p.detach().t())


@pytest.mark.parametrize("overlap", ["1", "0"])
def test_optimizer_clears_the_gradients_it_consumed(gpu, monkeypatch, overlap):
    """Eager GPU steps: the fused Adam clears each gradient slice it reads and the next step skips its memset. After
    every step the whole gradient buffer is zero, and the losses track a trainer that zeroes with a separate memset
    (same init, same batches; not bitwise: the backward's fp32 atomics sum in a run-dependent order)."""
    from huggingface_sagemaker_tensorflow_distributed_amd import data as hdata
    from huggingface_sagemaker_tensorflow_distributed_amd.train.runner import build
    from huggingface_sagemaker_tensorflow_distributed_amd.utils.args import build_parser

    ds = hdata.synthetic_classification(8 * 4, 128, 30522, seed=0)
    batches = [{k: torch.from_numpy(v[8 * i:8 * (i + 1)]).long().to(gpu) for k, v in
                (("input_ids", ds.input_ids), ("attention_mask", ds.attention_mask), ("labels", ds.labels))}
               for i in range(4)]
    monkeypatch.setenv("HSD_OPT_OVERLAP", overlap)
    losses = {}
    for zero_in_opt in (True, False):
        # a small learning rate: at 1e-4 this tiny-batch run is unstable (loss 0.8 -> 2.8 in a step) and run-to-run
        # atomics noise grows to 2e-3 within 4 steps with or without the zeroing
        args, _ = build_parser("train").parse_known_args(
            ["--model_name_or_path", "bert-base-uncased", "--train_batch_size", "8", "--learning_rate", "2e-5",
             "--dtype", "bf16", "--log_every", "0", "--hip_graph", "false", "--seed", "3",
             "--gradient_accumulation_steps", "2"])
        parts = build(args, "train")
        tr, st = parts["trainer"], parts["store"]
        tr.zero_grad_in_optimizer = zero_in_opt
        assert (tr._opt_overlap is not None) == (overlap == "1")
        out = []
        for step in range(4):
            out.append(float(tr.train_step([batches[(2 * step + j) % 4] for j in range(2)])))
            torch.cuda.synchronize()
            if zero_in_opt:
                assert tr._grads_clear and int(torch.count_nonzero(st.grad)) == 0
        losses[zero_in_opt] = out
    a, b = losses[True], losses[False]
    assert a[0] == b[0]
    for x, y in zip(a, b):
        assert abs(x - y) <= 2e-3 * max(1.0, abs(y)), (a, b)


def test_two_layer_bert_learns_the_marker_task(gpu, tmp_path):
    """End-to-end learning on the HIP path: a 2-layer bert-base-width model from random init learns the synthetic
    marker task (label carried by one token at a random position of a padded sequence) to > 95 % held-out accuracy
    (tools/convergence.py runs the 12-layer version against the torch reference)."""
    import json

    from huggingface_sagemaker_tensorflow_distributed_amd import data as hdata
    from huggingface_sagemaker_tensorflow_distributed_amd.data.loader import BatchLoader
    from huggingface_sagemaker_tensorflow_distributed_amd.parallel import ShardSampler
    from huggingface_sagemaker_tensorflow_distributed_amd.train.runner import build
    from huggingface_sagemaker_tensorflow_distributed_amd.utils.args import build_parser

    cfg = {"model_type": "bert", "vocab_size": 30522, "hidden_size": 768, "num_hidden_layers": 2,
           "num_attention_heads": 12, "intermediate_size": 3072, "max_position_embeddings": 512, "type_vocab_size": 2,
           "num_labels": 2}
    (tmp_path / "config.json").write_text(json.dumps(cfg))
    args, _ = build_parser("train").parse_known_args(
        ["--model_name_or_path", str(tmp_path), "--train_batch_size", "32", "--learning_rate", "1e-4",
         "--dtype", "bf16", "--log_every", "0", "--hip_graph", "false", "--seed", "7"])
    parts = build(args, "train")
    tr = parts["trainer"]
    ds = hdata.synthetic_classification(32 * 300, 128, 30522, seed=1)
    for i in range(300):
        sl = slice(32 * i, 32 * (i + 1))
        tr.train_step([{k: torch.from_numpy(v[sl]).long().to(gpu) for k, v in
                        (("input_ids", ds.input_ids), ("attention_mask", ds.attention_mask), ("labels", ds.labels))}])
    test = hdata.synthetic_classification(512, 128, 30522, seed=2)
    ev = tr.evaluate(BatchLoader(test, ShardSampler(512, 0, 1, shuffle=False, drop_last=False, batch_size=64), gpu))
    assert ev["sparse_categorical_accuracy"] > 0.95, ev


def test_small_step_without_stored_wt_matches_with(gpu, monkeypatch):
    """bert-large at the reference's own per-rank shape class (B = 2, S = 512: under the Wᵀ token threshold): the
    store without Wᵀ copies (dgrads read W directly) trains exactly like the store with them -- same losses and
    the same weights after 3 steps (the two dgrad layouts are bit-identical)."""
    from huggingface_sagemaker_tensorflow_distributed_amd.optim import FusedAdam
    from huggingface_sagemaker_tensorflow_distributed_amd.parallel import FlatParamStore
    from huggingface_sagemaker_tensorflow_distributed_amd.train.trainer import Trainer

    monkeypatch.setenv("HSD_OPT_OVERLAP", "0")
    cfg = resolve_config("bert-large-uncased").replace(num_hidden_layers=2, hidden_dropout_prob=0.0,
                                                        attention_probs_dropout_prob=0.0)
    g = torch.Generator().manual_seed(0)
    batches = [{"input_ids": torch.randint(5, cfg.vocab_size, (2, 512), generator=g).to(gpu),
                "attention_mask": torch.ones(2, 512, dtype=torch.long, device=gpu),
                "labels": torch.randint(0, 2, (2,), generator=g).to(gpu)} for _ in range(3)]
    runs = []
    for keep in (True, False):
        m = build_model(cfg, seed=0).to(gpu)
        store = FlatParamStore(m, gpu, compute_dtype=torch.bfloat16, transposed=keep)
        assert (store.transposed is not None) == keep
        tr = Trainer(m, store, FusedAdam(store, lr=1e-4), None, gpu)
        losses = [float(tr.train_step([b]).detach()) for b in batches]
        torch.cuda.synchronize()
        runs.append((losses, store.master.clone()))
    (l0, m0), (l1, m1) = runs
    assert l0[0] == l1[0]
    assert max(abs(a - b) for a, b in zip(l0, l1)) < 1e-3, (l0, l1)
    assert float((m0 - m1).abs().max()) < 1e-3


def test_fp32_mode_on_gpu_matches_cpu_fp32(gpu, tmp_path):
    """--dtype fp32 (the reference's precision, scripts/train.py:113-123) trains on the GPU -- fp32 reference ops,
    fused fp32 Adam -- and reproduces the CPU fp32 run of the same job (same seeds, data, dropout masks): the epoch
    loss / accuracy and the eval metrics agree to fp32 summation-order noise."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = {}
    for device in ("cuda", "cpu"):
        d = tmp_path / device
        env = dict(os.environ, SM_OUTPUT_DATA_DIR=str(d / "data"), SM_MODEL_DIR=str(d / "model"), SM_NUM_GPUS="1",
                   SM_FRAMEWORK_PARAMS="{}")
        cmd = [sys.executable, os.path.join(root, "scripts", "train.py"), "--epochs", "1", "--train_batch_size", "8",
               "--eval_batch_size", "8", "--model_name_or_path", "hsd-tiny-bert", "--max_seq_length", "64",
               "--num_train_examples", "64", "--num_eval_examples", "32", "--dtype", "fp32", "--device", device,
               "--log_every", "0", "--hip_graph", "false"]
        r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
        assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
        ev = dict(line.split(" = ") for line in (d / "data" / "eval_results.txt").read_text().splitlines())
        tr = (d / "data" / "train_results.txt").read_text().splitlines()[0]
        out[device] = (float(ev["loss"]), float(ev["sparse_categorical_accuracy"]), float(tr.split("[")[1].split("]")[0]))
    (gl, ga, gt), (cl, ca, ct) = out["cuda"], out["cpu"]
    assert abs(gl - cl) < 1e-3 * max(1.0, abs(cl)), (gl, cl)
    assert abs(gt - ct) < 1e-3 * max(1.0, abs(ct)), (gt, ct)
    assert abs(ga - ca) <= 1.0 / 32 + 1e-9, (ga, ca)
