"""HIP-graph replay of the training step (train/graph.py) vs the same steps run eagerly.

Both trainers use graph-mode seeding (fixed per-site seeds + the device step seed), so dropout masks are
identical and the only difference is capture/replay: losses and weights must agree to rounding
(fp32 atomics in the backward reduce in a different order between runs)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _trainer(gpu, graph_replay, **kw):
    from huggingface_sagemaker_tensorflow_distributed_amd.models import build_model, resolve_config
    from huggingface_sagemaker_tensorflow_distributed_amd.optim import FusedAdam
    from huggingface_sagemaker_tensorflow_distributed_amd.parallel import FlatParamStore
    from huggingface_sagemaker_tensorflow_distributed_amd.train.trainer import Trainer

    cfg = resolve_config("bert-base-uncased").replace(num_hidden_layers=2)
    model = build_model(cfg, seed=0).to(gpu)
    model.rng.base_seed = 5
    store = FlatParamStore(model, gpu, compute_dtype=torch.bfloat16)
    opt = FusedAdam(store, lr=1e-4, weight_decay=kw.pop("weight_decay", 0.0))
    tr = Trainer(model, store, opt, None, gpu, hip_graph=True, **kw)
    tr._graph_replay = graph_replay
    return tr


@pytest.mark.parametrize("full", ["1", "0"])
def test_graph_replay_matches_eager(gpu, monkeypatch, full):
    """full=1: the whole step (zeroing, fwd, bwd, overlapped Adam slices, Wᵀ refresh) is one graph replay with
    device-side Adam scalars; full=0: fwd+bwd graph, eager optimizer. Both with the weight-gradient side stream as a
    branch of the graph. A linear LR schedule with warm-up and AdamW
    weight decay make every step's scalars differ."""
    monkeypatch.setenv("HSD_GRAPH_FULL", full)
    g = torch.Generator().manual_seed(0)
    batches = []
    for _ in range(3):
        ids = torch.randint(1000, 30000, (16, 128), generator=g)
        am = torch.ones(16, 128, dtype=torch.long)
        am[3, 70:] = 0
        batches.append({"input_ids": ids.to(gpu), "attention_mask": am.to(gpu),
                        "labels": torch.randint(0, 2, (16,), generator=g).to(gpu)})
    from huggingface_sagemaker_tensorflow_distributed_amd.ops import hip

    res = {}
    for replay in (False, True):
        tr = _trainer(gpu, replay, weight_decay=0.01, lr_schedule="linear", lr_warmup_steps=2)
        tr.total_steps = 3
        side0 = hip.CAPTURES_WITH_SIDE_STREAM[0]
        losses = [float(tr.train_step([b])) for b in batches]
        if replay:
            assert len(tr._graphs) == 1
            assert tr._full_graph == (full == "1")
            # 2048-token steps run their weight gradients on the side stream: a branch of the captured graph
            assert hip.CAPTURES_WITH_SIDE_STREAM[0] == side0 + 1
        assert tr.optimizer.step_count == 3
        torch.cuda.synchronize()
        res[replay] = (losses, tr.store.master.clone())
        tr._seed.close()
    (l0, w0), (l1, w1) = res[False], res[True]
    for a, b in zip(l0, l1):
        assert abs(a - b) <= 2e-3 * max(1.0, abs(a)), (l0, l1)
    rel = (w0 - w1).norm() / w0.norm()
    assert rel < 1e-4, float(rel)
    # dropout masks move with the step: the three losses are not a replay of one step
    assert len({round(x, 6) for x in l1}) == 3


def test_graph_accumulation_and_metrics_match_eager(gpu, monkeypatch):
    """Two accumulation micro-steps (fwd+bwd graph per micro-step, optimizer slices stepped at the join) and the
    fused-head metrics of graph replays (static output buffers: every step's stats are kept, not the last one's)."""
    from huggingface_sagemaker_tensorflow_distributed_amd.train.trainer import _Meter

    g = torch.Generator().manual_seed(1)
    mbs = []
    for _ in range(4):
        ids = torch.randint(1000, 30000, (8, 128), generator=g)
        mbs.append({"input_ids": ids.to(gpu), "attention_mask": torch.ones(8, 128, dtype=torch.long, device=gpu),
                    "labels": torch.randint(0, 2, (8,), generator=g).to(gpu)})
    res = {}
    for replay in (False, True):
        tr = _trainer(gpu, replay)
        meter = _Meter(gpu)
        tr.train_step(mbs[:2], meter)
        tr.train_step(mbs[2:], meter)
        m = meter.result(global_=False)
        torch.cuda.synchronize()
        res[replay] = (m, tr.store.master.clone())
        tr._seed.close()
    (m0, w0), (m1, w1) = res[False], res[True]
    assert (w0 - w1).norm() / w0.norm() < 1e-4
    for k in m0:
        assert abs(m0[k] - m1[k]) <= 2e-3 * max(1.0, abs(m0[k])), (m0, m1)

    # one-micro-step graph replays: metrics over 2 steps = eager metrics
    monkeypatch.setenv("HSD_GRAPH_FULL", "1")
    res = {}
    for replay in (False, True):
        tr = _trainer(gpu, replay)
        meter = _Meter(gpu)
        tr.train_step(mbs[:1], meter)
        tr.train_step(mbs[1:2], meter)
        res[replay] = meter.result(global_=False)
        tr._seed.close()
    for k in res[False]:
        assert abs(res[False][k] - res[True][k]) <= 2e-3 * max(1.0, abs(res[False][k])), res


def test_eval_graph_and_coalescing_match_eager(gpu):
    """``Trainer.evaluate`` by captured-forward replays (``eval_hip_graph``, one graph per batch shape) == the eager
    forwards, and coalesced eval batches (runner ``--eval_coalesce_tokens``: k batches of 2 per forward) give the same
    per-example metrics as one forward per batch of 2 -- the reference's eval_batch_size 2 (launch.py:16)."""
    from huggingface_sagemaker_tensorflow_distributed_amd.train.graph import CapturedEval  # noqa: F401

    g = torch.Generator().manual_seed(3)
    n, S = 24, 128
    ids = torch.randint(1000, 30000, (n, S), generator=g)
    am = torch.ones(n, S, dtype=torch.long)
    am[5, 60:] = 0
    am[17, 90:] = 0
    labels = torch.randint(0, 2, (n,), generator=g)

    def batches(bs):
        return [{"input_ids": ids[i:i + bs].to(gpu), "attention_mask": am[i:i + bs].to(gpu),
                 "labels": labels[i:i + bs].to(gpu)} for i in range(0, n, bs)]

    tr = _trainer(gpu, True)
    tr._seed.close()
    res = {}
    for flag in (False, True):
        tr.eval_hip_graph = flag
        res[flag] = tr.evaluate(batches(2))
        assert tr.eval_graph_active == flag
    assert len(tr._eval_graphs) == 1  # one shape, captured once
    assert res[False] == res[True], res  # the same kernels replayed: identical sums
    tr.eval_hip_graph = True
    big = tr.evaluate(batches(8))  # 4 batches of 2 per forward
    assert abs(big["loss"] - res[True]["loss"]) <= 1e-3 * abs(res[True]["loss"]), (big, res[True])
    assert abs(big["sparse_categorical_accuracy"] - res[True]["sparse_categorical_accuracy"]) <= 1.0 / n + 1e-9
