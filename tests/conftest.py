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


def _refresh_native_knobs():
    """The native launchers cache their HSD_* knobs (csrc/kernels/common.h HSD_KNOB); re-read them when a test changes
    the environment. No-op unless the extension is already loaded (CPU tier)."""
    mod = sys.modules.get("huggingface_sagemaker_tensorflow_distributed_amd._C") or sys.modules.get(
        "huggingface_sagemaker_tensorflow_distributed_amd._C_debug")
    if mod is not None and hasattr(mod, "refresh_env"):
        mod.refresh_env()


@pytest.fixture(autouse=True)
def _native_knobs(monkeypatch):
    # every test starts from the (already undone) environment of the previous one; knob flips inside the test go
    # through monkeypatch.setenv / delenv, which re-read the cache at once
    _refresh_native_knobs()
    set0, del0 = monkeypatch.setenv, monkeypatch.delenv

    def setenv(name, value, prepend=None):
        set0(name, value, prepend)
        _refresh_native_knobs()

    def delenv(name, raising=True):
        del0(name, raising)
        _refresh_native_knobs()

    monkeypatch.setenv, monkeypatch.delenv = setenv, delenv
    yield
