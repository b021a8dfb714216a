"""Deterministic mode (utils/determinism.py): two runs from the same seed agree bitwise --
on the PyTorch path and on the fused HIP path (its fixed-order reduction forms); without the mode the
fused path (a few float-atomic reductions) agrees to rounding."""
import pytest
import torch

from proteinbert_pytorch_replication_amd.data import SyntheticUniRefGO
from proteinbert_pytorch_replication_amd.models import ProteinBERT
from proteinbert_pytorch_replication_amd.train.optim import FusedAdam
from proteinbert_pytorch_replication_amd.train.step import PretrainStep
from proteinbert_pytorch_replication_amd.utils import determinism


def _run(device, backend, steps=3, L=64, A=96, G=64, C=32, B=6, blocks=2, semantics="reference"):
    torch.manual_seed(0)
    m = ProteinBERT(sequences_length=L, num_annotations=A, local_dim=C, global_dim=G,
                    key_dim=64 if C == 128 else 16, num_heads=4, num_blocks=blocks, device=device, backend=backend,
                    semantics=semantics)
    opt = FusedAdam(m.parameters(), lr=1e-3)
    step = PretrainStep(m, opt)
    gen = SyntheticUniRefGO(L, A, B, device, seed=7)
    losses = [float(step(*gen.next_batch())) for _ in range(steps)]
    if device.type == "cuda":
        torch.cuda.synchronize()
    return losses, torch.cat([p.detach().reshape(-1).float().cpu() for p in m.parameters()])


def _enable_and_restore():
    prev = torch.are_deterministic_algorithms_enabled()
    determinism.enable()
    return prev


def test_deterministic_mode_bitwise_cpu():
    prev = _enable_and_restore()
    try:
        dev = torch.device("cpu")
        assert determinism.fused_deterministic()
        l1, p1 = _run(dev, "torch")
        l2, p2 = _run(dev, "torch")
    finally:
        torch.use_deterministic_algorithms(prev)
        determinism._STATE["on"] = False
    assert l1 == l2
    assert torch.equal(p1, p2)


@pytest.mark.gpu
@pytest.mark.parametrize("L,B,blocks", [(128, 8, 2), (512, 16, 6)])
def test_deterministic_mode_bitwise_fused_hip(L, B, blocks):
    """The fused HIP step twice from the same seed: every loss and every parameter bitwise equal
    (L = 128 < 2 x CUs exercises the LayerNorm-affine single-writer form; the paper config at L = 512)."""
    prev = _enable_and_restore()
    try:
        dev = torch.device("cuda")
        assert determinism.backend_for("hip") == "hip"
        l1, p1 = _run(dev, "hip", L=L, A=8943, G=512, C=128, B=B, blocks=blocks)
        l2, p2 = _run(dev, "hip", L=L, A=8943, G=512, C=128, B=B, blocks=blocks)
    finally:
        torch.use_deterministic_algorithms(prev)
        determinism._STATE["on"] = False
    print("max |dp| between runs:", float((p1 - p2).abs().max()))
    assert l1 == l2
    assert torch.equal(p1, p2)


@pytest.mark.gpu
def test_hip_path_reproducible_to_rounding():
    """Fused path (local_dim 128), default (atomic) forms: same seed twice, the float-atomic reduction
    order may differ; the run-to-run parameter difference is bounded and reported."""
    dev = torch.device("cuda")
    l1, p1 = _run(dev, "hip", L=128, A=256, G=256, C=128, B=8)
    l2, p2 = _run(dev, "hip", L=128, A=256, G=256, C=128, B=8)
    for a, b in zip(l1, l2):
        assert abs(a - b) <= 1e-4 * abs(a)
    # Adam normalises updates: bound the parameter drift by the step count x lr
    print("max |dp| between runs (atomic forms):", float((p1 - p2).abs().max()))
    assert float((p1 - p2).abs().max()) <= 3 * 2 * 1e-3


def test_cli_deterministic_flag_reproduces_losses(tmp_path, capsys):
    """``kernel.deterministic=true`` from the pretrain CLI: two fresh runs give identical losses."""
    import json
    from proteinbert_pytorch_replication_amd.cli.train import pretrain_main
    small = ["model.sequences_length=32", "model.num_annotations=40", "model.local_dim=16", "model.global_dim=32",
             "model.key_dim=8", "model.num_blocks=1", "train.batch_size=4", "kernel.dtype=fp32",
             "kernel.deterministic=true", "train.max_batch_iterations=3", "train.nb_iterations_checkpoint=100"]
    prev = torch.are_deterministic_algorithms_enabled()
    outs = []
    try:
        for i in range(2):
            pretrain_main(["--preset", "cfg1_cpu_smoke", *small, f"train.save_path={tmp_path}/r{i}",
                           "--resume", "none"])
            outs.append(json.loads(capsys.readouterr().out.strip().splitlines()[-1]))
    finally:
        torch.use_deterministic_algorithms(prev)
        determinism._STATE["on"] = False
    assert outs[0]["final_loss"] == outs[1]["final_loss"]


def test_backend_routing_without_fixed_order_kernels():
    """Deterministic mode keeps its bitwise guarantee for configurations whose HIP kernels only have
    float-atomic reductions (paper semantics, non-fused global-track shapes): they run on the PyTorch
    path; reference semantics at the fused shapes stay on HIP."""
    from proteinbert_pytorch_replication_amd.config import get_preset
    prev = torch.are_deterministic_algorithms_enabled()
    try:
        assert determinism.backend_for("hip", {"semantics": "paper"}) == "hip"      # mode off: request stands
        determinism.enable()
        cfg = get_preset("cfg2_paper_l512").model
        assert determinism.backend_for("hip", cfg) == "hip"
        assert determinism.backend_for("hip", dict(semantics="paper", global_dim=512, local_dim=128)) == "torch"
        assert determinism.backend_for("auto", dict(semantics="reference", global_dim=384, local_dim=128)) == "torch"
        assert determinism.backend_for("torch", dict(semantics="paper")) == "torch"
    finally:
        determinism.disable()
        torch.use_deterministic_algorithms(prev)


def test_model_routes_itself_under_determinism():
    """the routing happens in ProteinBERT.resolved_backend on the model's own config, so a
    paper-semantics model built with backend='auto' or 'hip' (bench.py, library users, a checkpoint
    loaded under another preset's flags) resolves to torch while the mode is on, and back to its request
    when it is off."""
    from proteinbert_pytorch_replication_amd.models import ProteinBERT
    prev = torch.are_deterministic_algorithms_enabled()
    cuda = torch.device("cuda")          # a device object only: resolved_backend never touches the GPU
    paper = ProteinBERT(16, 20, 32, 64, 8, 2, 1, semantics="paper", backend="hip", device="cpu")
    ref = ProteinBERT(16, 20, 128, 512, 8, 4, 1, semantics="reference", backend="hip", device="cpu")
    try:
        assert paper.resolved_backend(cuda) == "hip"
        determinism.enable()
        assert paper.resolved_backend(cuda) == "torch"
        paper.backend = "auto"
        assert paper.resolved_backend(cuda) == "torch"
        assert ref.resolved_backend(cuda) == "hip"           # fixed-order kernels exist: stays on HIP
    finally:
        determinism.disable()
        torch.use_deterministic_algorithms(prev)
    assert paper.resolved_backend(torch.device("cpu")) == "torch"


def test_deterministic_paper_semantics_bitwise_cpu():
    """Paper semantics in deterministic mode: routed to the PyTorch path (its HIP kernels reduce with float
    atomics), and two runs from the same seed agree bitwise."""
    prev = _enable_and_restore()
    try:
        dev = torch.device("cpu")
        be = determinism.backend_for("hip", dict(semantics="paper", global_dim=64, local_dim=32))
        assert be == "torch"
        l1, p1 = _run(dev, be, semantics="paper")
        l2, p2 = _run(dev, be, semantics="paper")
    finally:
        torch.use_deterministic_algorithms(prev)
        determinism._STATE["on"] = False
    assert l1 == l2
    assert torch.equal(p1, p2)
