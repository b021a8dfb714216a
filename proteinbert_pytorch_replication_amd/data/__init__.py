"""Data layer: vocabulary, transforms, datasets, on-disk store, synthetic on-device batches."""
from .vocab import (Vocab, create_amino_acid_vocab, ALL_AMINO_ACIDS, SPECIAL_TOKENS, PAD_ID, SOS_ID,
                    EOS_ID, UNK_ID, VOCAB_SIZE)
from .transforms import (SimpleCharacterTokenizer, SentenceRandomCrop, SimpleTokenRandomizer,
                         AnnotationMasking, pad_to)
from .datasets import (UniRefGO_PretrainingDataset, UniRefGO_StorePretrainingDataset,
                       UniRefGO_HDF5PretrainingDataset, collate_triples)
from .store import ProteinStore, ProteinStoreWriter, has_h5py
from .synthetic import (SyntheticUniRefGO, MultiLengthSynthetic, CorruptionParams, corrupt_batch_torch,
                        create_random_samples)

__all__ = [n for n in dir() if not n.startswith("_")]
