"""--hip_graph auto: the replay is chosen only for launch-bound single-process GPU steps (runner.resolve_hip_graph)."""
import pytest

from huggingface_sagemaker_tensorflow_distributed_amd.train.runner import resolve_hip_graph
from huggingface_sagemaker_tensorflow_distributed_amd.utils.args import bool_or_auto


def test_flag_parses_auto_and_booleans():
    assert bool_or_auto("auto") == "auto" and bool_or_auto("AUTO") == "auto"
    assert bool_or_auto("true") is True and bool_or_auto("0") is False
    with pytest.raises(Exception):
        bool_or_auto("sometimes")


@pytest.mark.parametrize("flag,on_gpu,world,tokens,accum,want", [
    ("auto", True, 1, 1024, 1, True),      # bert-base S=128 B=8
    ("auto", True, 1, 2048, 1, True),      # B=16: the measured crossover
    ("auto", True, 1, 4096, 1, False),     # B=32 / bert-large B=8: eager wins
    ("auto", True, 2, 1024, 1, False),     # data parallel: whole-step DP capture stays opt-in
    ("auto", True, 1, 1024, 2, False),     # gradient accumulation
    ("auto", False, 1, 1024, 1, False),    # CPU
    (True, False, 1, 10 ** 6, 4, True),    # explicit flags pass through
    (False, True, 1, 128, 1, False),
])
def test_resolve(flag, on_gpu, world, tokens, accum, want, monkeypatch):
    monkeypatch.delenv("HSD_GRAPH_AUTO_MAX_TOKENS", raising=False)
    assert resolve_hip_graph(flag, on_gpu, world, tokens, accum) is want


def test_cap_env(monkeypatch):
    monkeypatch.setenv("HSD_GRAPH_AUTO_MAX_TOKENS", "8192")
    assert resolve_hip_graph("auto", True, 1, 4096, 1) is True
