"""Model families: ProteinBERT pretraining model and fine-tuning heads."""
from .proteinbert import ProteinBERT, ProteinBERTBlock, GlobalAttention, GlobalAttentionHead, build_model
from .finetune import ProteinBERTForTokenClassification, ProteinBERTForSequenceClassification

__all__ = ["ProteinBERT", "ProteinBERTBlock", "GlobalAttention", "GlobalAttentionHead", "build_model",
           "ProteinBERTForTokenClassification", "ProteinBERTForSequenceClassification"]
