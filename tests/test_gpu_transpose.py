"""Batched bf16 weight transpose (transpose_many: the dgrad GEMMs' Wᵀ copies, parallel/flat_params.py) against
torch's transpose, for full 64 x 64 tiles (16-B path) and edge tiles (dimensions that are multiples of 4 only)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("shapes", [
    [(768, 2304), (768, 768), (3072, 768), (768, 3072)],
    [(100, 36), (64, 64), (12, 8), (136, 200), (4, 4)],
    [(1024, 4096), (72, 1032)],
])
def test_transpose_many_matches_torch(gpu, shapes):
    from huggingface_sagemaker_tensorflow_distributed_amd.ops import hip
    srcs = [torch.randn(r, c, device=gpu).bfloat16() for r, c in shapes]
    dsts = [torch.full((c, r), 7.0, device=gpu, dtype=torch.bfloat16) for r, c in shapes]
    desc, tiles = [], 0
    for s, d in zip(srcs, dsts):
        r, c = s.shape
        desc.append([s.data_ptr(), d.data_ptr(), r, c, tiles])
        tiles += ((r + 63) // 64) * ((c + 63) // 64)
    hip._C.transpose_many(torch.tensor(desc, dtype=torch.int64, device=gpu), tiles)
    torch.cuda.synchronize()
    for s, d in zip(srcs, dsts):
        assert torch.equal(d, s.t()), s.shape
