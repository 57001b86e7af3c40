"""Launch modes and failure handling on CPU / gloo (SURVEY.md §4 'dist', §5 failure detection):

* ``scripts/singe_node_train.py`` under the launcher keeps MirroredStrategy semantics (GLOBAL batch split over the
  ranks, no ``train_runtime`` line; reference ``scripts/singe_node_train.py:17,96-101``);
* the ``HuggingFace`` estimator look-alike with an ``smdistributed`` distribution spawns one rank per process slot and
  writes the reference artifacts (reference ``launch.py:20,36-55``);
* an injected fault on one rank (``HSD_FAULT_RANK`` / ``HSD_FAULT_STEP``) fails the whole job with a non-zero code;
* an injected HANG on one rank (``HSD_FAULT_HANG=1``) is turned into a failed job by ``--step_watchdog`` within its
  timeout (the stalled rank, and the rank blocked in the all-reduce behind it, exit non-zero; the launcher tears down);
* ``--check_sync`` detects ranks whose parameters diverged.
"""
import io
import os
import socket
import sys

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.dist

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
TINY = ["--model_name_or_path", "hsd-tiny-bert", "--epochs", "1", "--max_seq_length", "32", "--num_train_examples", "64",
        "--num_eval_examples", "32", "--device", "cpu", "--log_every", "0"]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_single_node_script_splits_global_batch(tmp_path):
    from huggingface_sagemaker_tensorflow_distributed_amd.launcher.spawn import launch

    buf = io.StringIO()
    rc = launch([sys.executable, os.path.join(ROOT, "scripts", "singe_node_train.py"), "--train_batch_size", "16",
                 "--eval_batch_size", "8"] + TINY + ["--benchmark", "True", "--warmup_steps", "1"], 2,
                output_data_dir=str(tmp_path / "data"), model_dir=str(tmp_path / "model"), stdout=buf)
    assert rc == 0, buf.getvalue()[-3000:]
    txt = (tmp_path / "data" / "train_results.txt").read_text()
    assert txt.startswith("loss = [") and "train_runtime" not in txt  # singe_node_train.py:96-101
    import json

    bench = json.load(open(tmp_path / "data" / "benchmark.json"))
    # global batch 16 over 2 replicas -> 8 sequences per rank per step
    assert bench.get("per_gpu_batch", bench.get("per_rank_batch")) == 8, bench
    assert (tmp_path / "model" / "model.safetensors").exists()


def test_estimator_smddp_distribution_runs_ranks(tmp_path, monkeypatch):
    from huggingface_sagemaker_tensorflow_distributed_amd.launcher.estimator import HuggingFace

    hp = {"epochs": 1, "train_batch_size": 8, "eval_batch_size": 8, "model_name_or_path": "hsd-tiny-bert",
          "max_seq_length": 32, "num_train_examples": 32, "num_eval_examples": 16, "device": "cpu", "log_every": 0}
    est = HuggingFace(entry_point="train.py", source_dir=os.path.join(ROOT, "scripts"), instance_type="local",
                      instance_count=1, distribution={"smdistributed": {"dataparallel": {"enabled": True}}},
                      hyperparameters=hp, nproc_per_node=2, output_path=str(tmp_path), role="ignored",
                      debugger_hook_config=False)
    assert est.fit() == 0
    out = os.path.join(str(tmp_path), est.latest_job_name)
    assert open(os.path.join(out, "output", "data", "eval_results.txt")).read().count(" = ") == 2
    assert os.path.exists(os.path.join(est.model_data, "config.json"))


def test_injected_fault_fails_the_job(tmp_path):
    from huggingface_sagemaker_tensorflow_distributed_amd.launcher.spawn import launch

    buf = io.StringIO()
    rc = launch([sys.executable, os.path.join(ROOT, "scripts", "train.py"), "--train_batch_size", "8",
                 "--eval_batch_size", "8"] + TINY, 2, output_data_dir=str(tmp_path / "data"),
                model_dir=str(tmp_path / "model"), env_extra={"HSD_FAULT_RANK": "1", "HSD_FAULT_STEP": "1"},
                stdout=buf, kill_grace_s=5)
    assert rc != 0, buf.getvalue()[-3000:]
    assert not (tmp_path / "model" / "model.safetensors").exists()


def test_injected_hang_is_caught_by_step_watchdog(tmp_path):
    import time

    from huggingface_sagemaker_tensorflow_distributed_amd.launcher.spawn import launch

    buf = io.StringIO()
    t0 = time.time()
    rc = launch([sys.executable, os.path.join(ROOT, "scripts", "train.py"), "--train_batch_size", "8",
                 "--eval_batch_size", "8", "--step_watchdog", "4"] + TINY, 2, output_data_dir=str(tmp_path / "data"),
                model_dir=str(tmp_path / "model"),
                env_extra={"HSD_FAULT_RANK": "1", "HSD_FAULT_STEP": "2", "HSD_FAULT_HANG": "1"},
                stdout=buf, kill_grace_s=5)
    elapsed = time.time() - t0
    log = buf.getvalue()
    assert rc != 0, log[-3000:]
    assert "step watchdog: rank" in log, log[-3000:]
    assert elapsed < 120, elapsed
    assert not (tmp_path / "model" / "model.safetensors").exists()


def _worker_sync(rank, world, port, q):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "LOCAL_WORLD_SIZE": str(world), "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    from huggingface_sagemaker_tensorflow_distributed_amd.models import build_model, resolve_config
    from huggingface_sagemaker_tensorflow_distributed_amd.optim import FusedAdam
    from huggingface_sagemaker_tensorflow_distributed_amd.parallel import (FlatParamStore, GradBucketer, backend,
                                                                           broadcast_parameters)
    from huggingface_sagemaker_tensorflow_distributed_amd.train.trainer import Trainer

    backend.init(device="cpu")
    cfg = resolve_config("hsd-tiny-bert").replace(hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
    model = build_model(cfg, seed=0)
    store = FlatParamStore(model, torch.device("cpu"))
    opt = FusedAdam(store, lr=1e-3)
    tr = Trainer(model, store, opt, GradBucketer(store, bucket_mb=0.05), torch.device("cpu"), check_sync=1)
    broadcast_parameters(store)
    g = torch.Generator().manual_seed(rank)
    batch = {"input_ids": torch.randint(5, 1024, (4, 16), generator=g),
             "attention_mask": torch.ones(4, 16, dtype=torch.long), "labels": torch.randint(0, 2, (4,), generator=g)}
    tr.train_step([batch])  # in sync: passes the check
    if rank == 1:
        with torch.no_grad():
            store.master[:10].add_(1.0)
    try:
        tr.train_step([batch])
        q.put((rank, "no error"))
    except RuntimeError as e:
        q.put((rank, str(e)))
    backend.shutdown()


def test_check_sync_detects_divergence():
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    mp.spawn(_worker_sync, args=(2, _port(), q), nprocs=2, join=True)
    got = dict(q.get() for _ in range(2))
    assert all("ranks diverged" in v for v in got.values()), got
