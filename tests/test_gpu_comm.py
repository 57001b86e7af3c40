"""Native RCCL CommEngine (csrc/comm/comm_engine.cpp) on one GPU: a world-of-one communicator exercises
the whole code path (event ordering, comm stream, bucket bookkeeping); multi-rank semantics are covered
by the gloo tests of the same GradBucketer and by the driver's multi-GPU run."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _C():
    from huggingface_sagemaker_tensorflow_distributed_amd.ops._ext import load

    return load()


def test_comm_engine_world_of_one(gpu):
    C = _C()
    uid = C.CommEngine.unique_id()
    assert isinstance(uid, bytes) and len(uid) == 128
    eng = C.CommEngine(0, 1, uid, gpu.index, True)
    assert eng.rank == 0 and eng.world == 1
    t = torch.arange(1000, dtype=torch.float32, device=gpu)
    eng.allreduce(t, True)
    assert torch.equal(t, torch.arange(1000, dtype=torch.float32, device=gpu))
    b = torch.randn(333, device=gpu).bfloat16()
    ref = b.clone()
    eng.broadcast(b, 0)
    assert torch.equal(b, ref)


def test_comm_engine_buckets(gpu):
    C = _C()
    eng = C.CommEngine(0, 1, C.CommEngine.unique_id(), gpu.index, True)
    flat = torch.randn(10_000, device=gpu)
    ref = flat.clone()
    # 3 buckets: params 0,1 -> b0; 2 -> b1; 3,4,5 -> b2
    eng.set_buckets(flat, [0, 4000, 5000], [4000, 5000, 10_000], [2, 1, 3], [0, 0, 1, 2, 2, 2])
    assert eng.num_buckets() == 3
    for step in range(2):
        eng.begin_step()
        assert eng.launched_count() == 0
        assert eng.mark_ready(0) == -1
        assert eng.mark_ready(2) == 1
        assert eng.mark_ready(1) == 0
        assert eng.launched_count() == 2
        eng.finish()  # launches bucket 2 (params 3-5 never arrived)
        assert eng.launched_count() == 3
    torch.cuda.synchronize()
    assert torch.equal(flat, ref)
    eng.begin_step()
    eng.mark_ready(2)
    with pytest.raises(RuntimeError):
        eng.mark_ready(2)


def test_hip_backward_through_native_engine(gpu):
    """Full bert-base HIP backward (fused blocks, task head, embeddings) driving the native engine: every
    bucket is launched exactly once DURING backward (no double readiness signal, no late gradient), and
    the world-of-one reduction leaves the gradients equal to a plain backward's."""
    from huggingface_sagemaker_tensorflow_distributed_amd import data as hdata
    from huggingface_sagemaker_tensorflow_distributed_amd.parallel import GradBucketer
    from huggingface_sagemaker_tensorflow_distributed_amd.train.runner import build
    from huggingface_sagemaker_tensorflow_distributed_amd.utils.args import build_parser

    args, _ = build_parser("train").parse_known_args(
        ["--model_name_or_path", "bert-base-uncased", "--train_batch_size", "16", "--dtype", "bf16",
         "--log_every", "0", "--hip_graph", "false"])
    parts = build(args, "train")
    model, store = parts["model"], parts["trainer"].store
    ds = hdata.synthetic_classification(16, 128, 30522, seed=0, full_length=True)
    ids, am, lab = (torch.from_numpy(v).long().to(gpu) for v in (ds.input_ids, ds.attention_mask, ds.labels))

    def grads(buck):
        store.zero_grad()
        model.rng.new_step(3)
        if buck is not None:
            buck.begin()
        loss, _ = model(ids, attention_mask=am, labels=lab)
        loss.backward()
        launched = None
        if buck is not None:
            launched = buck.engine.launched_count()
            buck.finish()
        torch.cuda.synchronize()
        return store.grad.clone(), launched

    ref, _ = grads(None)
    C = _C()
    eng = C.CommEngine(0, 1, C.CommEngine.unique_id(), gpu.index, True)
    buck = GradBucketer(store, bucket_mb=16, engine=eng)
    assert eng.num_buckets() > 4
    for _ in range(2):
        g, launched = grads(buck)
        assert launched == eng.num_buckets()
        rel = (g - ref).norm() / ref.norm()
        assert rel < 1e-2, rel
    # overlap timeline: every bucket but the tail ones starts before backward ends
    assert buck.set_timing(True)
    grads(buck)
    rep = buck.overlap_report()
    buck.set_timing(False)
    assert rep is not None and len(rep["buckets"]) == eng.num_buckets()
    assert rep["backward_ms"] > 0 and rep["bytes"] == store.grad.numel() * 4
    assert all(0 <= s <= e for s, e, _ in rep["buckets"])
    assert sum(s < rep["backward_ms"] for s, _, _ in rep["buckets"]) >= eng.num_buckets() - 2
    buck.detach()


def test_optimizer_overlap_on_engine_stream(gpu, monkeypatch):
    """DP form of the optimizer overlap: each bucket's Adam slice runs on the RCCL engine's stream right after the
    bucket's all-reduce (world-of-one communicator here). Every step must equal one full Adam pass over that step's
    final (reduced) gradients, bit for bit."""
    from huggingface_sagemaker_tensorflow_distributed_amd import data as hdata
    from huggingface_sagemaker_tensorflow_distributed_amd.ops import hip
    from huggingface_sagemaker_tensorflow_distributed_amd.parallel import GradBucketer
    from huggingface_sagemaker_tensorflow_distributed_amd.train.runner import build
    from huggingface_sagemaker_tensorflow_distributed_amd.train.trainer import Trainer
    from huggingface_sagemaker_tensorflow_distributed_amd.utils.args import build_parser

    monkeypatch.setenv("HSD_OPT_OVERLAP", "1")
    args, _ = build_parser("train").parse_known_args(
        ["--model_name_or_path", "bert-base-uncased", "--train_batch_size", "8", "--dtype", "bf16",
         "--learning_rate", "1e-4", "--log_every", "0", "--hip_graph", "false"])
    parts = build(args, "train")
    model, store, opt = parts["model"], parts["store"], parts["optimizer"]
    C = _C()
    eng = C.CommEngine(0, 1, C.CommEngine.unique_id(), gpu.index, True)
    buck = GradBucketer(store, bucket_mb=4, engine=eng)
    tr = Trainer(model, store, opt, buck, gpu)
    tr.zero_grad_in_optimizer = False  # the replay below reads the step's reduced gradients after the step
    assert tr._opt_overlap == "engine" and len(opt._ranges) == len(buck.buckets) > 10
    ds = hdata.synthetic_classification(16, 128, 30522, seed=0)
    batches = [{k: torch.from_numpy(v[8 * i:8 * (i + 1)]).long().to(gpu) for k, v in
                (("input_ids", ds.input_ids), ("attention_mask", ds.attention_mask), ("labels", ds.labels))}
               for i in range(2)]
    for step in range(3):
        p0, m0, v0 = store.master.clone(), opt.exp_avg.clone(), opt.exp_avg_sq.clone()
        tr.train_step([batches[step % 2]])
        torch.cuda.synchronize()
        assert eng.launched_count() == len(buck.buckets)
        s, eps = opt._coeffs()
        out = torch.empty_like(store.compute)
        hip.adam_step(p0, m0, v0, store.grad, out, None, s, eps, opt.beta1, opt.beta2, 1.0, 0.0)
        torch.cuda.synchronize()
        assert torch.equal(p0, store.master) and torch.equal(m0, opt.exp_avg) and torch.equal(v0, opt.exp_avg_sq)
        assert torch.equal(out, store.compute)


def test_engine_optimizer_slices_clear_gradients(gpu, monkeypatch):
    """DP form of the gradient zeroing: the engine-stream Adam slices clear every gradient they consumed, so after each
    step the whole buffer is zero and the next step skips its memset; the losses track the same steps with a memset
    per step (world-of-one communicator; not bitwise: fp32 atomics in the backward)."""
    from huggingface_sagemaker_tensorflow_distributed_amd import data as hdata
    from huggingface_sagemaker_tensorflow_distributed_amd.parallel import GradBucketer
    from huggingface_sagemaker_tensorflow_distributed_amd.train.runner import build
    from huggingface_sagemaker_tensorflow_distributed_amd.train.trainer import Trainer
    from huggingface_sagemaker_tensorflow_distributed_amd.utils.args import build_parser

    monkeypatch.setenv("HSD_OPT_OVERLAP", "1")
    ds = hdata.synthetic_classification(16, 128, 30522, seed=0)
    batches = [{k: torch.from_numpy(v[8 * i:8 * (i + 1)]).long().to(gpu) for k, v in
                (("input_ids", ds.input_ids), ("attention_mask", ds.attention_mask), ("labels", ds.labels))}
               for i in range(2)]
    C = _C()
    losses = {}
    for zero_in_opt in (True, False):
        args, _ = build_parser("train").parse_known_args(
            ["--model_name_or_path", "bert-base-uncased", "--train_batch_size", "8", "--dtype", "bf16",
             "--learning_rate", "2e-5", "--log_every", "0", "--hip_graph", "false", "--seed", "3"])
        parts = build(args, "train")
        model, store, opt = parts["model"], parts["store"], parts["optimizer"]
        eng = C.CommEngine(0, 1, C.CommEngine.unique_id(), gpu.index, True)
        buck = GradBucketer(store, bucket_mb=4, engine=eng)
        tr = Trainer(model, store, opt, buck, gpu)
        tr.zero_grad_in_optimizer = zero_in_opt
        assert tr._opt_overlap == "engine"
        out = []
        for step in range(3):
            out.append(float(tr.train_step([batches[step % 2]])))
            torch.cuda.synchronize()
            if zero_in_opt:
                assert tr._grads_clear and int(torch.count_nonzero(store.grad)) == 0
        losses[zero_in_opt] = out
        buck.detach()
    a, b = losses[True], losses[False]
    assert a[0] == b[0]
    for x, y in zip(a, b):
        assert abs(x - y) <= 2e-3 * max(1.0, abs(y)), (a, b)


@pytest.mark.parametrize("mode,dtype", [(1, torch.bfloat16), (2, torch.float16)])
def test_comm_engine_wire_compression(gpu, mode, dtype):
    """set_compression (Horovod's hvd.Compression.fp16): each fp32 bucket is cast to 16 bits on the comm stream,
    all-reduced, cast back. With a world of one the result is the 16-bit rounding of the gradients, bucket by
    bucket, including the bucket finish() launches; a bad mode is refused."""
    C = _C()
    eng = C.CommEngine(0, 1, C.CommEngine.unique_id(), gpu.index, True)
    flat = torch.randn(10_000, device=gpu)
    ref = flat.to(dtype).float()
    eng.set_buckets(flat, [0, 4000, 5000], [4000, 5000, 10_000], [2, 1, 3], [0, 0, 1, 2, 2, 2])
    eng.set_compression(mode)
    eng.begin_step()
    assert eng.mark_ready(2) == 1
    eng.mark_ready(0)
    eng.mark_ready(1)
    eng.finish()
    torch.cuda.synchronize()
    assert torch.equal(flat, ref)
    with pytest.raises(RuntimeError):
        eng.set_compression(3)


def test_whole_step_graph_with_native_engine(gpu, monkeypatch):
    """Data-parallel whole-step HIP graph (train/graph.py CapturedTrainStep): the bucket all-reduces and the Adam slices
    on the engine stream are captured with forward / backward (world-of-one RCCL communicator). Three replayed steps
    equal three eager steps of the same engine configuration (same dropout masks via graph-mode seeding)."""
    from huggingface_sagemaker_tensorflow_distributed_amd import data as hdata
    from huggingface_sagemaker_tensorflow_distributed_amd.parallel import GradBucketer
    from huggingface_sagemaker_tensorflow_distributed_amd.train.runner import build
    from huggingface_sagemaker_tensorflow_distributed_amd.train.trainer import Trainer
    from huggingface_sagemaker_tensorflow_distributed_amd.utils.args import build_parser

    monkeypatch.setenv("HSD_OPT_OVERLAP", "1")
    monkeypatch.setenv("HSD_GRAPH_FULL", "1")
    monkeypatch.setenv("HSD_GRAPH_DP", "1")  # data-parallel whole-step capture is opt-in
    ds = hdata.synthetic_classification(32, 128, 30522, seed=1)
    batches = [{k: torch.from_numpy(v[16 * i:16 * (i + 1)]).long().to(gpu) for k, v in
                (("input_ids", ds.input_ids), ("attention_mask", ds.attention_mask), ("labels", ds.labels))}
               for i in range(2)]
    res = {}
    C = _C()
    for replay in (False, True):
        args, _ = build_parser("train").parse_known_args(
            ["--model_name_or_path", "bert-base-uncased", "--train_batch_size", "16", "--dtype", "bf16",
             "--learning_rate", "1e-4", "--log_every", "0", "--hip_graph", "false", "--seed", "3"])
        parts = build(args, "train")
        model, store, opt = parts["model"], parts["store"], parts["optimizer"]
        model.cfg  # noqa: B018
        eng = C.CommEngine(0, 1, C.CommEngine.unique_id(), gpu.index, True)
        buck = GradBucketer(store, bucket_mb=8, engine=eng)
        tr = Trainer(model, store, opt, buck, gpu, hip_graph=True)
        tr._graph_replay = replay
        assert tr._opt_overlap == "engine" and tr._seed is not None
        losses = [float(tr.train_step([batches[s % 2]])) for s in range(3)]
        torch.cuda.synchronize()
        if replay:
            assert any(k[0] == "full" for k in tr._graphs)
        assert opt.step_count == 3
        res[replay] = (losses, store.master.clone())
        tr._seed.close()
        buck.detach()
        eng.close()  # its teardown syncs and frees: not from a garbage collection inside the next capture
    (l0, w0), (l1, w1) = res[False], res[True]
    for a, b in zip(l0, l1):
        assert abs(a - b) <= 2e-3 * max(1.0, abs(a)), (l0, l1)
    assert float((w0 - w1).norm() / w0.norm()) < 1e-4


def test_whole_step_graph_waits_for_delayed_wgrad_branch(gpu, monkeypatch):
    """Ordering inside the data-parallel whole-step capture: the side stream is stalled 4 ms before each backward's
    first weight gradient (ops/hip.py HSD_TEST_SIDE_DELAY_US), so a bucket all-reduce / Adam slice that is ordered only
    after the capture stream reads main_grad before the wgrad branch has written it. The engine must wait on the wgrad
    branch once the capture has forked it (comm_engine.cpp set_capture_deps): replayed steps then equal eager steps."""
    from huggingface_sagemaker_tensorflow_distributed_amd import data as hdata
    from huggingface_sagemaker_tensorflow_distributed_amd.ops import hip
    from huggingface_sagemaker_tensorflow_distributed_amd.parallel import GradBucketer
    from huggingface_sagemaker_tensorflow_distributed_amd.train.runner import build
    from huggingface_sagemaker_tensorflow_distributed_amd.train.trainer import Trainer
    from huggingface_sagemaker_tensorflow_distributed_amd.utils.args import build_parser

    monkeypatch.setenv("HSD_OPT_OVERLAP", "1")
    monkeypatch.setenv("HSD_GRAPH_FULL", "1")
    monkeypatch.setenv("HSD_GRAPH_DP", "1")
    monkeypatch.setattr(hip, "_SIDE_DELAY_US", 4000.0)
    ds = hdata.synthetic_classification(32, 128, 30522, seed=2)
    batches = [{k: torch.from_numpy(v[16 * i:16 * (i + 1)]).long().to(gpu) for k, v in
                (("input_ids", ds.input_ids), ("attention_mask", ds.attention_mask), ("labels", ds.labels))}
               for i in range(2)]
    res = {}
    C = _C()
    for replay in (False, True):
        args, _ = build_parser("train").parse_known_args(
            ["--model_name_or_path", "bert-base-uncased", "--train_batch_size", "16", "--dtype", "bf16",
             "--learning_rate", "1e-4", "--log_every", "0", "--hip_graph", "false", "--seed", "5"])
        parts = build(args, "train")
        model, store, opt = parts["model"], parts["store"], parts["optimizer"]
        eng = C.CommEngine(0, 1, C.CommEngine.unique_id(), gpu.index, True)
        buck = GradBucketer(store, bucket_mb=4, engine=eng)
        tr = Trainer(model, store, opt, buck, gpu, hip_graph=True)
        tr._graph_replay = replay
        assert tr._opt_overlap == "engine"
        n0 = hip.CAPTURES_WITH_SIDE_STREAM[0]
        losses = [float(tr.train_step([batches[s % 2]])) for s in range(3)]
        torch.cuda.synchronize()
        if replay:
            assert any(k[0] == "full" for k in tr._graphs)
            assert hip.CAPTURES_WITH_SIDE_STREAM[0] > n0  # the capture really branched the wgrad side stream
        res[replay] = (losses, store.master.clone())
        tr._seed.close()
        buck.detach()
        eng.close()  # its teardown syncs and frees: not from a garbage collection inside the next capture
    (l0, w0), (l1, w1) = res[False], res[True]
    for a, b in zip(l0, l1):
        assert abs(a - b) <= 2e-3 * max(1.0, abs(a)), (l0, l1)
    assert float((w0 - w1).norm() / w0.norm()) < 1e-4
