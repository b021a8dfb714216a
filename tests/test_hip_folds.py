"""GPU: the fixed-order column-sum folds (csrc/glob.hip colsum_add / colsum_add2) vs fp64 torch sums."""
import pytest
import torch

from proteinbert_pytorch_replication_amd.ops import _lib
from proteinbert_pytorch_replication_amd.ops import local_track  # noqa: F401  (registers the launchers)

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("rows", [1, 7, 96, 257])
def test_colsum_add_pair_matches_torch(rows):
    dev = torch.device("cuda")
    c0, c1 = 128 * 128, 128
    slab = torch.randn(rows * (c0 + c1), device=dev)
    d0 = torch.randn(c0, device=dev)
    d1 = torch.randn(c1, device=dev)
    r0 = d0.double() + slab[:rows * c0].view(rows, c0).double().sum(0)
    r1 = d1.double() + slab[rows * c0:].view(rows, c1).double().sum(0)
    _lib.call("pbx_colsum_add2", slab.data_ptr(), c0, d0.data_ptr(), slab[rows * c0:].data_ptr(), c1, d1.data_ptr(),
              rows, _lib.stream_ptr(dev))
    torch.cuda.synchronize()
    assert (d0.double() - r0).abs().max().item() < 1e-4 * max(1.0, rows ** 0.5)
    assert (d1.double() - r1).abs().max().item() < 1e-4 * max(1.0, rows ** 0.5)
    # same order as two colsum_add launches: bitwise equal
    e0 = torch.zeros(c0, device=dev)
    e1 = torch.zeros(c1, device=dev)
    f0 = torch.zeros(c0, device=dev)
    f1 = torch.zeros(c1, device=dev)
    st = _lib.stream_ptr(dev)
    _lib.call("pbx_colsum_add2", slab.data_ptr(), c0, e0.data_ptr(), slab[rows * c0:].data_ptr(), c1, e1.data_ptr(),
              rows, st)
    _lib.call("pbx_colsum_add", slab.data_ptr(), rows, c0, f0.data_ptr(), None, st)
    _lib.call("pbx_colsum_add", slab[rows * c0:].data_ptr(), rows, c1, f1.data_ptr(), None, st)
    torch.cuda.synchronize()
    assert torch.equal(e0, f0) and torch.equal(e1, f1)
