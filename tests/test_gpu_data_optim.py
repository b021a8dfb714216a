"""GPU: fused Adam, on-device synthetic generation and corruption kernels vs torch oracles."""
import pytest
import torch

from proteinbert_pytorch_replication_amd.ops import _lib
from proteinbert_pytorch_replication_amd.data.synthetic import CorruptionParams, corrupt_batch_torch
from proteinbert_pytorch_replication_amd.train.optim import FusedAdam

pytestmark = pytest.mark.gpu


def test_hip_library_loads():
    assert _lib.available()
    _lib.lib()


def test_fused_adam_gpu_matches_torch():
    torch.manual_seed(0)
    shapes = [(129, 7), (1000,), (3, 5, 9), (1,)]
    ps = [torch.nn.Parameter(torch.randn(s, device="cuda")) for s in shapes]
    ref = [torch.nn.Parameter(p.detach().clone()) for p in ps]
    fa = FusedAdam(ps, lr=3e-3, weight_decay=0.1)
    ta = torch.optim.Adam(ref, lr=3e-3, weight_decay=0.1)
    for _ in range(6):
        grads = [torch.randn_like(p) for p in ps]
        fa.zero_grad()
        for p, g in zip(ps, grads):
            p.grad.copy_(g)
        fa.step()
        ta.zero_grad()
        for p, g in zip(ref, grads):
            p.grad = g.clone()
        ta.step()
    torch.cuda.synchronize()
    for p, r in zip(ps, ref):
        torch.testing.assert_close(p.detach(), r.detach(), rtol=2e-6, atol=2e-6)


def test_fused_adam_skip_flag():
    p = torch.nn.Parameter(torch.ones(100, device="cuda"))
    fa = FusedAdam([p], lr=0.1)
    p.grad.fill_(1.0)
    fa.skip_flag = torch.ones(1, dtype=torch.int32, device="cuda")
    fa.step()
    assert torch.all(p.detach() == 1.0)
    fa.skip_flag = torch.zeros(1, dtype=torch.int32, device="cuda")
    fa.step()
    assert torch.all(p.detach() < 1.0)


@pytest.mark.parametrize("n", [1, 7, 4096, 300001])
def test_nonfinite_flag_kernel(n):
    """pbx_nonfinite_flag: 1 iff any gradient element is NaN / Inf (every position, tail included)."""
    p = torch.nn.Parameter(torch.zeros(n, device="cuda"))
    fa = FusedAdam([p], lr=0.1)
    p.grad.copy_(torch.randn(n, device="cuda") * 1e30)          # huge but finite: not flagged
    assert int(fa.set_nonfinite_skip().item()) == 0
    for bad in (float("inf"), float("-inf"), float("nan")):
        for pos in sorted({0, n // 2, n - 1}):
            g = torch.randn(n, device="cuda")
            g[pos] = bad
            p.grad.copy_(g)
            assert int(fa.set_nonfinite_skip().item()) == 1, (bad, pos)
    p.grad.zero_()
    assert int(fa.set_nonfinite_skip().item()) == 0


@pytest.mark.parametrize("n", [5, 300001])
def test_nonfinite_flag_bound_and_accumulate(n):
    """The DP form: bound = FLT_MAX / world flags finite elements whose sum over the ranks could overflow, and
    accumulate = 1 ORs into the flag (one flag per step over every bucket)."""
    from proteinbert_pytorch_replication_amd.ops import _lib
    ws = torch.empty(1024, dtype=torch.int32, device="cuda")
    flag = torch.zeros(1, dtype=torch.int32, device="cuda")
    st = _lib.stream_ptr(torch.device("cuda"))
    bound = 3.4028234663852886e38 / 8
    g = torch.randn(n, device="cuda")

    def run(x, acc):
        _lib.call("pbx_nonfinite_flag", x.data_ptr(), x.numel(), ws.data_ptr(), flag.data_ptr(), bound, acc, st)
        return int(flag.item())

    assert run(g, 0) == 0
    big = g.clone()
    big[n - 1] = 5e37                           # finite, but 8 ranks of it overflow fp32
    assert run(big, 0) == 1
    assert run(g, 1) == 1                       # accumulate keeps the earlier bucket's 1
    assert run(g, 0) == 0                       # a fresh step overwrites
    ok = g.clone()
    ok[0] = 3e37                                # below FLT_MAX / 8
    assert run(ok, 1) == 0
    nan = g.clone()
    nan[n // 2] = float("nan")
    assert run(nan, 1) == 1


def test_clip_grad_norm_gpu():
    p = torch.nn.Parameter(torch.zeros(5000, device="cuda"))
    fa = FusedAdam([p], lr=0.1)
    p.grad.copy_(torch.randn(5000, device="cuda"))
    ref = p.grad.detach().clone()
    norm = fa.clip_grad_norm_(1.0)
    torch.testing.assert_close(norm, ref.norm(), rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(p.grad.norm(), torch.tensor(1.0, device="cuda"), rtol=1e-3, atol=1e-3)


@pytest.mark.parametrize("grad_scale", [0.5, 0.125])
def test_clip_grad_norm_gpu_grad_scale(grad_scale):
    """Under DP the arena holds the SUM gradient and grad_scale=1/world turns it into the mean: the
    HIP clip must match the CPU branch and torch's clip_grad_norm_ applied to grad*grad_scale."""
    torch.manual_seed(1)
    g0 = torch.randn(7001) * 3.0
    p = torch.nn.Parameter(torch.zeros(7001, device="cuda"))
    fa = FusedAdam([p], lr=0.1)
    fa.grad_scale = grad_scale
    p.grad.copy_(g0.cuda())
    norm = fa.clip_grad_norm_(1.0)
    # CPU branch of the same optimizer
    q = torch.nn.Parameter(torch.zeros(7001))
    fc = FusedAdam([q], lr=0.1, bf16_shadow=False)
    fc.grad_scale = grad_scale
    q.grad.copy_(g0)
    norm_c = fc.clip_grad_norm_(1.0)
    # torch oracle on the mean gradient
    r = torch.nn.Parameter(torch.zeros(7001))
    r.grad = g0 * grad_scale
    norm_t = torch.nn.utils.clip_grad_norm_([r], 1.0)
    torch.testing.assert_close(norm.cpu(), norm_t, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(torch.as_tensor(norm_c).float(), norm_t, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close((p.grad * grad_scale).cpu(), r.grad, rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(p.grad.cpu(), q.grad, rtol=1e-4, atol=1e-6)


def test_synth_and_corrupt_kernels():
    from proteinbert_pytorch_replication_amd.ops.corrupt import synth_batch, corrupt_batch
    B, L, A = 512, 128, 2000
    tok, ann = synth_batch(B, L, A, 0, 250, 0.01, seed=7, step=1, device="cuda")
    # structure: rows start with <sos> unless cropped; pads only at the tail
    is_pad = tok == 0
    assert torch.all(is_pad[:, 1:] >= is_pad[:, :-1])
    assert tok.min() >= 0 and tok.max() <= 25
    assert abs(ann.mean().item() - 0.01) < 0.002
    p = CorruptionParams()
    X, Y, W = corrupt_batch(tok, ann, p, seed=7, step=1)
    Xr, Yr, Wr = corrupt_batch_torch(tok, ann, p)
    # exact parts
    assert torch.equal(W["local"], Wr["local"])
    assert torch.equal(W["global"], Wr["global"])
    special = tok <= 2
    assert torch.equal(X["local"][special], tok[special])
    # statistical parts
    eligible = (~special).sum().item()
    changed = (X["local"] != tok).sum().item()
    # corruption rate p * P(new != old) = 0.05 * 22/23
    assert abs(changed / eligible - 0.05 * 22 / 23) < 0.01
    blank = (X["global"].sum(1) == 0) & (ann.sum(1) > 0)
    assert 0.4 < blank.float().mean().item() < 0.6
    kept = X["global"][~blank][ann[~blank] > 0]
    assert abs((kept > 0).float().mean().item() - 0.75) < 0.05


def test_native_loader_gpu_expansion_matches_cpu(tmp_path):
    """Compact loader batches expanded by pbx_unpack_batch == the NumPy expansion."""
    import numpy as np
    from proteinbert_pytorch_replication_amd.data.native_loader import NativeStoreLoader
    from proteinbert_pytorch_replication_amd.data.store import ProteinStoreWriter
    rng = np.random.default_rng(1)
    A = 8943
    path = str(tmp_path / "g.pbxds")
    w = ProteinStoreWriter(path, ["a%d" % i for i in range(A)])
    for i in range(70):
        w.append_mask("p%d" % i, "".join(rng.choice(list("ACDEFGHIKLMNPQRSTVWY"), int(rng.integers(5, 700)))),
                      rng.random(A) < 0.01)
    w.close()
    g = NativeStoreLoader(path, 16, 512, device="cuda", seed=4)
    c = NativeStoreLoader(path, 16, 512, device="cpu", seed=4)
    for _ in range(6):
        Xg, Yg, Wg = g.next_batch()
        Xc, Yc, Wc = c.next_batch()
        torch.cuda.synchronize()
        assert torch.equal(Yg["local"].cpu(), Yc["local"])
        assert torch.equal(Yg["global"].cpu(), Yc["global"])
        assert torch.equal(Wg["local"].cpu(), Wc["local"])
        assert torch.equal(Wg["global"].cpu(), Wc["global"])
        special = Yg["local"] <= 2
        assert torch.equal(Xg["local"][special], Yg["local"][special])
    g.close()
    c.close()
