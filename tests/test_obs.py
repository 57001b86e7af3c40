"""Observability: throughput meter, metrics.jsonl, benchmark.json and the profiler trace on CPU."""
import json
import os

from huggingface_sagemaker_tensorflow_distributed_amd.train.runner import run


def test_benchmark_and_profile_outputs(tmp_path, monkeypatch):
    monkeypatch.setenv("SM_OUTPUT_DATA_DIR", str(tmp_path / "data"))
    monkeypatch.setenv("SM_MODEL_DIR", str(tmp_path / "model"))
    out = run(["--model_name_or_path", "hsd-tiny-bert", "--epochs", "1", "--train_batch_size", "4",
               "--num_train_examples", "48", "--num_eval_examples", "8", "--max_seq_length", "32",
               "--benchmark", "True", "--profile", "True", "--warmup_steps", "2", "--log_every", "4",
               "--device", "cpu", "--do_eval", "False"], mode="train")
    d = tmp_path / "data"
    bench = json.loads((d / "benchmark.json").read_text())
    assert bench["n_gpus"] == 1 and bench["per_gpu_batch"] == 4 and bench["seq_len"] == 32
    assert bench["timed_steps"] == 12 - 1 - 2 and bench["value"] > 0
    lines = [json.loads(x) for x in (d / "metrics.jsonl").read_text().splitlines()]
    assert lines and all(r["ms_per_step"] > 0 for r in lines)
    assert os.path.getsize(d / "trace_rank0.json") > 0 and (d / "kernels_rank0.txt").exists()
    assert "history" in out
