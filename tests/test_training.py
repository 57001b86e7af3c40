"""Trainer-level behaviour on CPU (SURVEY.md §4 'unit / CPU', §5 checkpoint/resume): resume equals
uninterrupted training, gradient accumulation equals the full batch, the MLM task end to end, and the
GPU-only switches (--dtype fp8, --hip_graph) degrading cleanly on CPU."""
import json
import os

import pytest
import torch

from huggingface_sagemaker_tensorflow_distributed_amd.models import build_model, resolve_config
from huggingface_sagemaker_tensorflow_distributed_amd.optim import FusedAdam
from huggingface_sagemaker_tensorflow_distributed_amd.parallel import FlatParamStore
from huggingface_sagemaker_tensorflow_distributed_amd.train.callbacks import load_checkpoint, save_checkpoint
from huggingface_sagemaker_tensorflow_distributed_amd.train.trainer import Trainer

CPU = torch.device("cpu")


def _trainer(dropout=0.1, seed=0, **kw):
    cfg = resolve_config("hsd-tiny-bert").replace(hidden_dropout_prob=dropout, attention_probs_dropout_prob=dropout)
    model = build_model(cfg, seed=seed)
    model.rng.base_seed = 7
    store = FlatParamStore(model, CPU)
    opt = FusedAdam(store, lr=1e-3)
    return Trainer(model, store, opt, None, CPU, **kw)


def _batches(n, B=8, S=16, seed=0):
    g = torch.Generator().manual_seed(seed)
    out = []
    for _ in range(n):
        am = torch.ones(B, S, dtype=torch.long)
        am[::3, S // 2:] = 0
        out.append({"input_ids": torch.randint(5, 1024, (B, S), generator=g), "attention_mask": am,
                    "labels": torch.randint(0, 2, (B,), generator=g)})
    return out


def test_checkpoint_resume_equals_uninterrupted(tmp_path):
    data = _batches(4)
    ref = _trainer()
    for b in data:
        ref.train_step([b])
    a = _trainer()
    for b in data[:2]:
        a.train_step([b])
    ck = str(tmp_path / "checkpoint-1")
    save_checkpoint(ck, a, epoch=1)
    assert sorted(os.listdir(ck)) == ["config.json", "model.safetensors", "optimizer.pt", "trainer_state.json"]
    assert json.load(open(os.path.join(ck, "trainer_state.json")))["global_step"] == 2
    b = _trainer(seed=123)  # different init: everything must come from the checkpoint
    st = load_checkpoint(ck, b)
    assert st["epoch"] == 1 and b.global_step == 2
    for x in data[2:]:
        b.train_step([x])
    torch.testing.assert_close(b.store.master, ref.store.master, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(b.optimizer.exp_avg_sq, ref.optimizer.exp_avg_sq, rtol=1e-5, atol=1e-9)


def test_gradient_accumulation_equals_full_batch():
    """k micro-steps of B/k == one step of B (dropout off: the masks of the two runs differ per call)."""
    full = _batches(1, B=8)[0]
    halves = [{k: v[:4] for k, v in full.items()}, {k: v[4:] for k, v in full.items()}]
    a = _trainer(dropout=0.0)
    a.train_step([full])
    b = _trainer(dropout=0.0, grad_accum=2)
    b.train_step(halves)
    torch.testing.assert_close(b.store.master, a.store.master, rtol=1e-5, atol=1e-6)


def test_dropout_masks_change_per_step_but_replay_within_step():
    tr = _trainer()
    b = _batches(1)[0]
    m = tr.model
    m.train()
    m.rng.new_step(3)
    l1 = m(b["input_ids"], attention_mask=b["attention_mask"], labels=b["labels"])[0]
    m.rng.new_step(3)
    l2 = m(b["input_ids"], attention_mask=b["attention_mask"], labels=b["labels"])[0]
    m.rng.new_step(4)
    l3 = m(b["input_ids"], attention_mask=b["attention_mask"], labels=b["labels"])[0]
    assert float(l1.detach()) == float(l2.detach()) and float(l1.detach()) != float(l3.detach())


def test_graph_step_seed_is_deterministic_and_varies():
    from huggingface_sagemaker_tensorflow_distributed_amd.train.graph import step_seed

    assert step_seed(7, 0, 5) == step_seed(7, 0, 5)
    seeds = {step_seed(7, r, s) for r in range(4) for s in range(64)}
    assert len(seeds) == 4 * 64
    assert all(0 <= w < 2 ** 32 for s in seeds for w in s)


def test_hip_graph_flag_stays_eager_on_cpu():
    tr = _trainer(hip_graph=True)
    assert tr._seed is None
    tr.train_step(_batches(1))


def _run_script(tmp_path, extra, monkeypatch):
    from huggingface_sagemaker_tensorflow_distributed_amd.train.runner import run

    d, m = tmp_path / "data", tmp_path / "model"
    monkeypatch.setenv("SM_OUTPUT_DATA_DIR", str(d))
    monkeypatch.setenv("SM_MODEL_DIR", str(m))
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        monkeypatch.delenv(k, raising=False)
    return run(["--epochs", "1", "--train_batch_size", "4", "--eval_batch_size", "4", "--max_steps", "2",
                "--num_train_examples", "16", "--num_eval_examples", "8", "--log_every", "0"] + extra), d, m


def test_masked_lm_task_end_to_end_cpu(tmp_path, monkeypatch):
    out, d, m = _run_script(tmp_path, ["--model_name_or_path", "hsd-tiny-roberta", "--task", "masked-lm",
                                       "--max_seq_length", "32"], monkeypatch)
    tr = open(d / "train_results.txt").read()
    assert tr.startswith("loss = [") and "sparse_categorical_accuracy = [" in tr
    cfg = json.load(open(m / "config.json"))
    assert cfg["architectures"] == ["RobertaForMaskedLM"]


def test_fp8_dtype_falls_back_to_bf16_on_cpu(tmp_path, monkeypatch):
    """--dtype fp8 is a GPU (HIP) feature; on CPU the run completes in bf16 with a warning."""
    out, d, m = _run_script(tmp_path, ["--model_name_or_path", "hsd-tiny-bert", "--dtype", "fp8",
                                       "--max_seq_length", "16"], monkeypatch)
    assert os.path.isfile(d / "eval_results.txt") and os.path.isfile(m / "model.safetensors")


def test_optimizer_overlap_slices_cover_store_in_backward_order():
    """The overlapped optimizer's slices (optim/adam.py plan_ranges): contiguous, 64-aligned, whole segments, in
    the store's backward layout order, covering every element exactly once."""
    from huggingface_sagemaker_tensorflow_distributed_amd.models import build_model, resolve_config
    from huggingface_sagemaker_tensorflow_distributed_amd.optim.adam import plan_ranges
    from huggingface_sagemaker_tensorflow_distributed_amd.parallel import FlatParamStore

    m = build_model(resolve_config("hsd-tiny-bert"), seed=0)
    store = FlatParamStore(m, "cpu")
    for mb in (0.001, 0.01, 1000.0):
        ranges, owner = plan_ranges(store, mb)
        assert ranges[0][0] == 0 and ranges[-1][1] == store.numel
        assert all(a[1] == b[0] for a, b in zip(ranges, ranges[1:]))
        assert all(s % 64 == 0 and e % 64 == 0 and e > s for s, e in ranges)
        assert owner == sorted(owner) and len(set(owner)) == len(ranges)
        for i, seg in enumerate(store.segments):
            s, e = ranges[owner[i]]
            assert s <= seg.offset and seg.offset + seg.numel <= e
    assert len(plan_ranges(store, 1000.0)[0]) == 1


def test_gemm_nt_split_policy(monkeypatch):
    """Small NT grids go to the 128 x 128 kernel (no K-splits); with it off, split-K only for NT grids that leave
    more than half of the 256 CUs idle, >= 8 K-tiles per split. Weight gradients: the cost model keeps the
    headline's split counts and takes 128 x 128 tiles where 256 x 256 tiles would need many thin splits."""
    from huggingface_sagemaker_tensorflow_distributed_amd.ops._ext import load

    C = load()
    assert C.gemm2_nt_splits(4096, 1024, 4096) == 1      # bert-large B=8 S=512: gemm2s, 256 tiles of 128^2
    assert C.gemm2_nt_splits(131072, 768, 768) == 1      # headline: 1536 tiles
    monkeypatch.setenv("HSD_G2_SMALL", "0")
    assert C.gemm2_nt_splits(4096, 1024, 4096) == 4      # 64 tiles of 256^2
    assert C.gemm2_nt_splits(4096, 768, 3072) == 5       # 48 tiles, 48 K-tiles
    assert C.gemm2_nt_splits(8192, 768, 768) == 1        # 96 tiles but only 12 K-tiles
    monkeypatch.delenv("HSD_G2_SMALL")
    assert C.gemm2_splits(2304, 768, 131072) == 9        # headline wgrads: 256^2 tiles, one wave of 256 CUs
    assert C.gemm2_splits(768, 768, 131072) == 28
    # small steps (4,096-8,192 tokens): the fewest 128^2 K-splits giving 384 workgroups (profiles/r6/
    # wgrad_min_grid_small_steps_r6.log); below 4,096 tokens 192
    assert C.gemm2_splits(1024, 1024, 4096) == 6
    assert C.gemm2_splits(3072, 1024, 4096) == 2         # 192 tiles -> 384 workgroups
    assert C.gemm2_splits(2304, 768, 8192) == 4          # 108 tiles -> 432 workgroups
    assert C.gemm2_splits(1024, 1024, 2048) == 3         # 64 tiles -> 192 workgroups
    assert C.gemm2_splits(3072, 1024, 2048) == 1         # 192 tiles: one split, accumulated in place
    monkeypatch.setenv("HSD_WGRAD_MIN_GRID", "0")        # the latency cost model at every size
    assert C.gemm2_splits(1024, 1024, 4096) == 4         # 128^2 tiles x 4 splits (256^2 would need 13+)


def test_tiny_bert_learns_the_marker_task_on_cpu():
    """The CPU (torch reference) path learns the synthetic marker task: the label is carried by one token at a
    random position of a padded, variable-length sequence (the GPU tier checks the same on the HIP kernels)."""
    import torch

    from huggingface_sagemaker_tensorflow_distributed_amd import data as hdata
    from huggingface_sagemaker_tensorflow_distributed_amd.train.runner import build
    from huggingface_sagemaker_tensorflow_distributed_amd.utils.args import build_parser

    args, _ = build_parser("train").parse_known_args(
        ["--model_name_or_path", "hsd-tiny-bert", "--train_batch_size", "16", "--learning_rate", "2e-3",
         "--log_every", "0", "--device", "cpu", "--seed", "7"])
    tr = build(args, "train")["trainer"]
    vocab = tr.model.cfg.vocab_size
    ds = hdata.synthetic_classification(16 * 100, 32, vocab, seed=1)
    losses = []
    for i in range(100):
        sl = slice(16 * i, 16 * (i + 1))
        losses.append(float(tr.train_step([{k: torch.from_numpy(v[sl]).long() for k, v in (
            ("input_ids", ds.input_ids), ("attention_mask", ds.attention_mask), ("labels", ds.labels))}]).detach()))
    assert sum(losses[:10]) / 10 > 0.5 and sum(losses[-20:]) / 20 < 0.2, losses[::10]


def test_lr_schedule_linear_warmup_decay():
    """--lr_schedule linear --lr_warmup_steps W: warmup to the base rate, then linear decay to 0; constant (the
    Keras reference) leaves the rate alone."""
    from huggingface_sagemaker_tensorflow_distributed_amd.models import build_model, resolve_config
    from huggingface_sagemaker_tensorflow_distributed_amd.optim import FusedAdam
    from huggingface_sagemaker_tensorflow_distributed_amd.parallel import FlatParamStore
    from huggingface_sagemaker_tensorflow_distributed_amd.train.trainer import Trainer

    m = build_model(resolve_config("hsd-tiny-bert"), seed=0)
    store = FlatParamStore(m, "cpu")
    tr = Trainer(m, store, FusedAdam(store, lr=1e-3), None, "cpu", lr_schedule="linear", lr_warmup_steps=2)
    tr.total_steps = 10
    lrs = [tr.lr_at(s) for s in range(10)]
    assert lrs[0] == 0.5e-3 and lrs[1] == 1e-3
    assert lrs[2] == 1e-3 and all(a > b for a, b in zip(lrs[2:], lrs[3:])) and abs(lrs[9] - 1e-3 / 8) < 1e-12
    const = Trainer(m, store, FusedAdam(store, lr=1e-3), None, "cpu")
    assert all(const.lr_at(s) == 1e-3 for s in range(5))


def test_failed_step_does_not_advance_adam_step_count():
    """an exception between begin_step (overlapped optimizer) and step() leaves step_count unchanged."""
    import torch

    from huggingface_sagemaker_tensorflow_distributed_amd.models import build_model, resolve_config
    from huggingface_sagemaker_tensorflow_distributed_amd.optim import FusedAdam
    from huggingface_sagemaker_tensorflow_distributed_amd.parallel import FlatParamStore

    m = build_model(resolve_config("hsd-tiny-bert"), seed=0)
    store = FlatParamStore(m, torch.device("cpu"))
    opt = FusedAdam(store, lr=1e-3)
    opt.enable_overlap([(0, store.numel)])
    opt.begin_step(grad_scale=1.0)
    assert opt.step_count == 1
    opt.abort_step()
    assert opt.step_count == 0 and not opt._began


def test_hvd_allreduce_average_rejects_integers_in_a_world_of_one():
    """the dtype check runs before the world-size early return (same error at any world size)."""
    import pytest
    import torch

    from huggingface_sagemaker_tensorflow_distributed_amd.parallel.collectives import hvd_allreduce

    with pytest.raises(TypeError):
        hvd_allreduce(torch.arange(4))
    assert torch.equal(hvd_allreduce(torch.arange(4), average=False), torch.arange(4))
