"""HIP-graph replay of the training step (train/graph.py) vs the same steps run eagerly.

Both trainers use graph-mode seeding (fixed per-site seeds + the device step seed), so dropout masks are
identical and the only difference is capture/replay: losses and weights must agree to rounding
(fp32 atomics in the backward reduce in a different order between runs)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _trainer(gpu, graph_replay):
    from huggingface_sagemaker_tensorflow_distributed_amd.models import build_model, resolve_config
    from huggingface_sagemaker_tensorflow_distributed_amd.optim import FusedAdam
    from huggingface_sagemaker_tensorflow_distributed_amd.parallel import FlatParamStore
    from huggingface_sagemaker_tensorflow_distributed_amd.train.trainer import Trainer

    cfg = resolve_config("bert-base-uncased").replace(num_hidden_layers=2)
    model = build_model(cfg, seed=0).to(gpu)
    model.rng.base_seed = 5
    store = FlatParamStore(model, gpu, compute_dtype=torch.bfloat16)
    opt = FusedAdam(store, lr=1e-4)
    tr = Trainer(model, store, opt, None, gpu, hip_graph=True)
    tr._graph_replay = graph_replay
    return tr


def test_graph_replay_matches_eager(gpu):
    g = torch.Generator().manual_seed(0)
    batches = []
    for _ in range(3):
        ids = torch.randint(1000, 30000, (16, 128), generator=g)
        am = torch.ones(16, 128, dtype=torch.long)
        am[3, 70:] = 0
        batches.append({"input_ids": ids.to(gpu), "attention_mask": am.to(gpu),
                        "labels": torch.randint(0, 2, (16,), generator=g).to(gpu)})
    res = {}
    for replay in (False, True):
        tr = _trainer(gpu, replay)
        losses = [float(tr.train_step([b])) for b in batches]
        if replay:
            assert len(tr._graphs) == 1
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
