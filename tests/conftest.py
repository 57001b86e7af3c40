import os
import sys

import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

os.environ.setdefault("HF_HUB_OFFLINE", "1")
os.environ.setdefault("TRANSFORMERS_OFFLINE", "1")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP kernels / RCCL)")
    config.addinivalue_line("markers", "dist: multi-process (gloo) test")
    config.addinivalue_line("markers", "slow: long-running test")
    config.addinivalue_line("markers", "multigpu: needs >= 2 GPUs on one node (skips cleanly otherwise)")


@pytest.fixture
def fake_sm_env(tmp_path, monkeypatch):
    d = tmp_path / "data"
    m = tmp_path / "model"
    monkeypatch.setenv("SM_OUTPUT_DATA_DIR", str(d))
    monkeypatch.setenv("SM_MODEL_DIR", str(m))
    monkeypatch.setenv("SM_NUM_GPUS", "0")
    monkeypatch.setenv("SM_FRAMEWORK_PARAMS", "{}")
    return {"data": str(d), "model": str(m)}


@pytest.fixture
def gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)
