"""GPU: the fused training step (reference semantics, synthetic on-device data, fused Adam) launches only
in-tree HIP kernels -- no PyTorch-native (at::native) kernel: the gradient-arena fill, the step counters,
the loss slots / total and the backward seed are in-tree or allocation-free (tools/native_ops.py is the
profiling probe at the bench shape).  Runtime copies / memsets are allowed and listed."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_fused_step_has_no_pytorch_native_kernels():
    from torch.profiler import ProfilerActivity, profile
    from proteinbert_pytorch_replication_amd.data import SyntheticUniRefGO
    from proteinbert_pytorch_replication_amd.models import ProteinBERT
    from proteinbert_pytorch_replication_amd.train.optim import FusedAdam
    from proteinbert_pytorch_replication_amd.train.step import PretrainStep
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = ProteinBERT(sequences_length=256, num_annotations=512, local_dim=128, global_dim=512, key_dim=64,
                    num_heads=4, num_blocks=2, device=dev, backend="hip")
    opt = FusedAdam(m.parameters(), lr=1e-3)
    step = PretrainStep(m, opt)
    gen = SyntheticUniRefGO(256, 512, 16, dev, seed=3)
    for _ in range(2):
        step(*gen.next_batch())
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        step(*gen.next_batch())
        torch.cuda.synchronize()
    names = [e.name for e in prof.events() if e.device_type.name == "CUDA"]
    assert len(names) > 20, names          # the profiler saw the step's kernels
    native = [n for n in names if "at::native" in n]
    assert not native, native
