"""GPU: the fixed-order column fold (csrc/glob.hip pbx_colsum_add / pbx_colsum_set).  Aligned inputs with a
column count divisible by 4 take the 16-B colsum_add4_kernel, anything else the scalar colsum_add_kernel;
both must give bitwise-equal sums (same per-column addition order), close to a float64 reference."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("rows,cols", [(256, 2 * 9 * 26 * 128), (7, 36), (56, 16388), (2, 8), (300, 3328)])
@pytest.mark.parametrize("fn", ["pbx_colsum_add", "pbx_colsum_set"])
def test_colsum_vector_path_bitwise(rows, cols, fn):
    from proteinbert_pytorch_replication_amd.ops import _lib, global_track  # noqa: F401  (registers)
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(rows * 7 + cols)
    src = torch.randn(rows * cols, device=dev, generator=g) * 3
    buf = torch.empty(rows * cols + 1, device=dev)
    buf[1:] = src
    src_mis = buf[1:]                      # 4-B offset: the scalar kernel
    assert src.data_ptr() % 16 == 0 and src_mis.data_ptr() % 16 != 0
    init = torch.randn(cols, device=dev, generator=g)
    dst_v, dst_s = init.clone(), init.clone()
    scale = torch.tensor([0.5], device=dev)
    st = _lib.stream_ptr(dev)
    _lib.call(fn, src.data_ptr(), rows, cols, dst_v.data_ptr(), scale.data_ptr(), st)
    _lib.call(fn, src_mis.data_ptr(), rows, cols, dst_s.data_ptr(), scale.data_ptr(), st)
    torch.cuda.synchronize()
    assert torch.equal(dst_v, dst_s)
    ref = src.double().view(rows, cols).sum(0) * 0.5
    if fn == "pbx_colsum_add":
        ref = ref + init.double()
    assert torch.allclose(dst_v.double(), ref, rtol=1e-5, atol=1e-4 * (rows ** 0.5))



@pytest.mark.parametrize("G,R,C", [(1024, 16, 128), (4096, 2, 64), (3, 1, 5)])
def test_group_colsum_in_order(G, R, C):
    from proteinbert_pytorch_replication_amd.ops.paper_track import group_colsum
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(G + R + C)
    src = torch.randn(G, R, C, device=dev, generator=g)
    out = group_colsum(src)
    ref = torch.zeros(G, C, device=dev)
    for r in range(R):                   # the kernel's order: r = 0 .. R-1, fp32
        ref = ref + src[:, r]
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
