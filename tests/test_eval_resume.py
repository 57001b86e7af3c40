"""Evaluation coverage, resume epoch accounting, loader failures and run provenance on CPU (SURVEY.md §4
'unit / CPU', §5 checkpoint/resume; round-1 advisor findings)."""
import json

import pytest
import torch

from huggingface_sagemaker_tensorflow_distributed_amd import data as hdata
from huggingface_sagemaker_tensorflow_distributed_amd.parallel.sampler import ShardSampler

from test_training import CPU, _run_script, _trainer


def test_resume_continues_epoch_count(tmp_path, monkeypatch):
    """--resume_from checkpoint-1 with --epochs 2 trains the ONE remaining epoch (Keras initial_epoch)."""
    common = ["--model_name_or_path", "hsd-tiny-bert", "--max_seq_length", "16", "--epochs", "2",
              "--max_steps", "0"]
    out, d, m = _run_script(tmp_path / "a", common + ["--save_every_epoch", "True"], monkeypatch)
    full_steps = out["global_step"]
    assert full_steps == 8 and len(out["history"]["loss"]) == 2  # 16 examples / batch 4 = 4 steps per epoch
    ck = m / "checkpoint-1"
    assert json.load(open(ck / "trainer_state.json"))["epoch"] == 1
    out2, _, _ = _run_script(tmp_path / "b", common + ["--resume_from", str(ck)], monkeypatch)
    assert len(out2["history"]["loss"]) == 1
    assert out2["global_step"] == full_steps


def test_eval_scores_every_example_once():
    """37 test examples at eval batch 8: the last partial batch counts (reference model.evaluate)."""
    tr = _trainer(dropout=0.0)
    ds = hdata.synthetic_classification(37, 16, 1024, seed=5)
    loader = hdata.BatchLoader(ds, ShardSampler(37, 0, 1, drop_last=False, mark_padding=True, batch_size=8), CPU)
    assert len(loader) == 5
    res = tr.evaluate(loader)
    ids = torch.from_numpy(ds.input_ids).long()
    am = torch.from_numpy(ds.attention_mask).long()
    lab = torch.from_numpy(ds.labels).long()
    tr.model.eval()
    with torch.no_grad():
        loss, logits = tr.model(ids, attention_mask=am, labels=lab)
    assert res["loss"] == pytest.approx(float(loss), rel=1e-5)
    assert res["sparse_categorical_accuracy"] == pytest.approx(float((logits.argmax(-1) == lab).float().mean()))


def test_padded_shards_mark_repeats_and_loader_ignores_them():
    n, world = 37, 4
    parts = [ShardSampler(n, r, world, drop_last=False, mark_padding=True).indices() for r in range(world)]
    assert len({len(p) for p in parts}) == 1
    assert sorted(i for p in parts for i in p if i >= 0) == list(range(n))  # every example exactly once
    assert sum(i < 0 for p in parts for i in p) == 3
    ds = hdata.synthetic_classification(n, 8, 512, seed=1)
    pad_rank = [r for r in range(world) if any(i < 0 for i in parts[r])][0]
    loader = hdata.BatchLoader(ds, ShardSampler(n, pad_rank, world, drop_last=False, mark_padding=True,
                                                batch_size=16), CPU)
    (b,) = list(loader)
    assert int((b["labels"] == -100).sum()) == 1 and b["num_valid"] == len(parts[pad_rank]) - 1


def test_loader_thread_failure_is_raised():
    ds = hdata.synthetic_classification(16, 8, 512, seed=1)
    loader = hdata.BatchLoader(ds, ShardSampler(16, 0, 1, batch_size=4), CPU)

    def boom(idx):
        raise ValueError("corrupt record")

    loader._host_batch = boom
    with pytest.raises(RuntimeError, match="prefetch") as ei:
        list(loader)
    assert isinstance(ei.value.__cause__, ValueError)


def test_synthetic_random_init_run_is_flagged(tmp_path, monkeypatch, capsys):
    _, d, _ = _run_script(tmp_path, ["--model_name_or_path", "hsd-tiny-bert", "--max_seq_length", "16"],
                          monkeypatch)
    prov = json.load(open(d / "run_provenance.json"))
    assert prov["synthetic_data"] is True and prov["weights"] == "random-init"
    log = capsys.readouterr()
    assert "WARNING - training on synthetic random data and random-init weights" in log.out + log.err
    assert open(d / "eval_results.txt").read().startswith("loss = ")  # the reference's format is untouched
