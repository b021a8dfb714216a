"""MI355X-native ProteinBERT pretraining / fine-tuning framework.

Capabilities of Aedelon/ProteinBERT-PyTorch-Replication (reference), rebuilt
for AMD Instinct MI355X (gfx950): PyTorch-ROCm for autograd glue and the
process group, hand-written CDNA4 HIP kernels for the hot ops (``ops/``),
RCCL over xGMI for data parallelism (``parallel/``).
"""
__version__ = "0.1.0"

from .config import (ModelConfig, DataConfig, OptimConfig, DistConfig, KernelConfig, TrainConfig,
                     RunConfig, PRESETS, get_preset, apply_overrides, load_yaml)
from .models import ProteinBERT, ProteinBERTBlock, GlobalAttention, build_model

__all__ = ["ModelConfig", "DataConfig", "OptimConfig", "DistConfig", "KernelConfig", "TrainConfig",
           "RunConfig", "PRESETS", "get_preset", "apply_overrides", "load_yaml", "ProteinBERT",
           "ProteinBERTBlock", "GlobalAttention", "build_model", "__version__"]
