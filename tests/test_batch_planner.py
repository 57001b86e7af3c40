"""``--train_batch_size auto``: per-GPU batch sized for the device memory (train/batch_planner.py).

CPU tier: the linear sizing rule, the analytic activation model, the CLI value and an end-to-end run of the entry
logic. GPU tier: the probe-based plan on one MI355X predicts the step's peak memory of the batch it picks.
"""
import json

import pytest
import torch

from huggingface_sagemaker_tensorflow_distributed_amd.models import resolve_config
from huggingface_sagemaker_tensorflow_distributed_amd.train import batch_planner as bp
from huggingface_sagemaker_tensorflow_distributed_amd.utils.args import parse_args

from test_training import _run_script


def test_choose_fits_budget_and_caps_tokens():
    GB = 2**30
    b, why = bp.choose(per_seq=40e6, fixed=5 * GB, budget=100 * GB, seq_len=128, max_tokens=None)
    assert why == "memory" and b % 8 == 0
    assert 5 * GB + 40e6 * b <= 100 * GB < 5 * GB + 40e6 * (b + 8)
    b, why = bp.choose(per_seq=40e6, fixed=5 * GB, budget=100 * GB, seq_len=128, max_tokens=131072)
    assert (b, why) == (1024, "max_tokens")
    b, why = bp.choose(per_seq=40e9, fixed=5 * GB, budget=10 * GB, seq_len=512)
    assert (b, why) == (1, "min")


def test_analytic_activation_model_scales_with_shape():
    base, large = resolve_config("bert-base-uncased"), resolve_config("bert-large-uncased")
    a = bp.activation_bytes_per_seq(base, 128)
    # bert-base S=128 keeps ~26 KB per token and layer in bf16: ~40 MB per sequence
    assert 30e6 < a < 50e6
    assert bp.activation_bytes_per_seq(base, 256) == pytest.approx(2 * a)
    assert bp.activation_bytes_per_seq(large, 128) > 2.5 * a


def test_cli_accepts_auto_and_keeps_int_default():
    args, _ = parse_args([])
    assert args.train_batch_size == 8 and isinstance(args.train_batch_size, int)
    args, _ = parse_args(["--train_batch_size", "auto"])
    assert args.train_batch_size == "auto"
    args, _ = parse_args(["--train_batch_size", "32"])
    assert args.train_batch_size == 32


def test_auto_batch_end_to_end_cpu(tmp_path, monkeypatch):
    """The entry logic resolves auto before building the loaders, trains at that batch and records the plan."""
    out, d, _ = _run_script(tmp_path, ["--model_name_or_path", "hsd-tiny-bert", "--max_seq_length", "16",
                                       "--train_batch_size", "auto", "--auto_batch_max_tokens", "64"], monkeypatch)
    prov = json.load(open(d / "run_provenance.json"))
    plan = prov["auto_batch"]
    assert plan["method"] == "analytic" and plan["capped_by"] == "max_tokens"
    assert plan["per_gpu_batch"] == 64 // 16 == prov["train_batch_size"]
    assert out["args"].train_batch_size == 4 and out["global_step"] == 2


def test_compression_shadow_counts_in_fixed_bytes():
    """--grad_compression fp16/bf16 adds the engine's 16-bit shadow of the fp32 gradient buffer (numel x 2 bytes),
    created after planning, to the planned fixed bytes."""
    from huggingface_sagemaker_tensorflow_distributed_amd.models import build_model
    from huggingface_sagemaker_tensorflow_distributed_amd.parallel import FlatParamStore

    model = build_model(resolve_config("hsd-tiny-bert"), seed=0)
    store = FlatParamStore(model, torch.device("cpu"))
    a = bp.plan(model, store, 16, "cpu", max_tokens=None)
    b = bp.plan(model, store, 16, "cpu", max_tokens=None, compression="fp16")
    assert b.fixed_bytes - a.fixed_bytes == store.numel * 2
    assert b.per_gpu_batch <= a.per_gpu_batch


@pytest.mark.gpu
def test_probe_plan_predicts_the_step_peak_on_gpu():
    """On the MI355X the two-probe linear model predicts the peak memory of a full training step (forward,
    backward, fused Adam) at the batch it picks, within 10 %, and the batch stays under the budget."""
    from huggingface_sagemaker_tensorflow_distributed_amd.models import build_model
    from huggingface_sagemaker_tensorflow_distributed_amd.optim import FusedAdam
    from huggingface_sagemaker_tensorflow_distributed_amd.parallel import FlatParamStore

    dev = torch.device("cuda", 0)
    cfg = resolve_config("bert-base-uncased").replace(num_hidden_layers=4)
    model = build_model(cfg, seed=0).to(dev)
    store = FlatParamStore(model, dev, compute_dtype=torch.bfloat16)
    opt = FusedAdam(store, lr=5e-5)
    S = 128
    # a small budget keeps the check fast: 12 GB over what the weights / optimizer already hold
    total = torch.cuda.mem_get_info(dev)[1]
    headroom = (torch.cuda.memory_allocated(dev) + 12 * 2**30) / total
    plan = bp.plan(model, store, S, dev, headroom=headroom, max_tokens=None)
    assert plan.method.startswith("probe") and plan.capped_by == "memory" and plan.per_gpu_batch >= 64, plan
    B = plan.per_gpu_batch
    ids = torch.randint(1000, cfg.vocab_size, (B, S), device=dev)
    am = torch.ones(B, S, dtype=torch.long, device=dev)
    labels = torch.randint(0, 2, (B,), device=dev)
    torch.cuda.synchronize(dev)
    torch.cuda.reset_peak_memory_stats(dev)
    model.train()
    model.rng.new_step(1)
    store.zero_grad()
    loss, _ = model(ids, attention_mask=am, labels=labels)
    loss.backward()
    opt.step(grad_scale=1.0)
    torch.cuda.synchronize(dev)
    peak = torch.cuda.max_memory_allocated(dev)
    assert torch.isfinite(loss).item()
    assert abs(peak - plan.predicted_peak_bytes) <= 0.10 * (peak - plan.fixed_bytes), (peak, plan)
    assert peak <= plan.budget_bytes * 1.02, (peak, plan)
