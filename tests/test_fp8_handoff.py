"""The producer -> consumer fp8 copy handoff (ops/hip.py _Q8Handoff): a copy is taken only by the
input that IS the producer's live, unmodified output, once. Pure host logic: runs on CPU tensors."""
import torch

from huggingface_sagemaker_tensorflow_distributed_amd.ops.hip import _Q8Handoff


def _copy(n):
    return torch.zeros(n, dtype=torch.uint8), torch.ones(1)


def test_taken_by_a_view_of_the_producer_output_once():
    h = _Q8Handoff()
    out = torch.randn(4, 8)
    q, s = _copy(32)
    h.put(out, q, s)
    got = h.take(out.view(32))  # the consumer reshapes: same memory, same size
    assert got is not None and got[0] is q and got[1] is s
    assert h.take(out) is None  # one consumer only


def test_not_taken_by_another_tensor_or_size():
    h = _Q8Handoff()
    out = torch.randn(4, 8)
    h.put(out, *_copy(32))
    assert h.take(torch.randn(4, 8)) is None
    h.put(out, *_copy(32))
    assert h.take(out[:2]) is None  # same start, different size


def test_not_taken_after_in_place_write():
    h = _Q8Handoff()
    out = torch.randn(4, 8)
    h.put(out, *_copy(32))
    out.mul_(2.0)  # the bf16 values no longer match the fp8 copy
    assert h.take(out) is None


def test_not_taken_after_producer_output_died():
    h = _Q8Handoff()
    out = torch.randn(1024)
    ptr = out.data_ptr()
    h.put(out, *_copy(1024))
    del out  # its memory may now back an unrelated tensor with the same address and size
    other = torch.empty(1024)
    assert h.take(other) is None, (ptr, other.data_ptr())
