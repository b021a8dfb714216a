"""Model families: ProteinBERT pretraining model and fine-tuning heads."""
from .proteinbert import ProteinBERT, ProteinBERTBlock, GlobalAttention, build_model

__all__ = ["ProteinBERT", "ProteinBERTBlock", "GlobalAttention", "build_model"]
