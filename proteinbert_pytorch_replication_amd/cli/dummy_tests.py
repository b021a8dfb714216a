"""Smoke driver with the reference's functions (``ProteinBERT/dummy_tests.py``, S1).

``create_random_samples`` / ``test_sequence_transform`` / ``test_sequence_token_randomizer`` /
``test_masking_annotation`` / ``test_data_processing`` print the data pipeline stages;
``main()`` builds the 100-sample DataFrame dataset (L=256, B=32), the paper model, prints its
summary and pretrains 250 iterations with Adam(lr=2e-4) - on the GPU through the fused HIP path.
torchtext is not used: the transforms are this package's equivalents; the reference's
``ToTensor(padding_value=seq_max_length)`` (pads with 128, a driver quirk) is reproduced for the
printout only.
"""
from __future__ import annotations

import argparse
import logging
import random
from typing import List, Optional, Sequence, Tuple

import pandas as pd
import torch
from torch.nn import BCELoss, CrossEntropyLoss
from torch.utils.data import DataLoader

from ..data import (AnnotationMasking, SentenceRandomCrop, SimpleCharacterTokenizer, SimpleTokenRandomizer,
                    UniRefGO_PretrainingDataset, collate_triples, create_amino_acid_vocab)
from ..data.vocab import ALL_AMINO_ACIDS
from ..models import ProteinBERT
from ..train.pretrain import pretrain
from ..utils.summary import summary

NB_ANNOTATIONS = 8943
NUM_WORKERS = 0
BATCH_SIZE = 32

Sample = Tuple[str, List[int]]


def create_random_samples(nb_samples: int, seed: int = 7777, nb_annotations: int = NB_ANNOTATIONS) -> List[Sample]:
    """Lengths U[0, 250], uniform amino acids, annotations Bernoulli(0.005) (same RNG stream as the
    reference: ``random.seed(seed)``, ``randint``/``random`` in the same order)."""
    random.seed(seed)
    samples = []
    for _ in range(nb_samples):
        n = random.randint(0, 250)
        seq = "".join(ALL_AMINO_ACIDS[random.randint(0, len(ALL_AMINO_ACIDS) - 1)] for _ in range(n))
        ann = [0 if random.random() * 1000 > 5 else 1 for _ in range(nb_annotations)]
        samples.append((seq, ann))
    return samples


def test_sequence_transform(samples: Sequence[Sample], vocab, seq_max_length: int):
    tok = SimpleCharacterTokenizer(vocab=vocab)
    crop = SentenceRandomCrop(max_length=seq_max_length)
    out = []
    for seq, ann in samples:
        out.append((torch.tensor(crop(tok(seq)), dtype=torch.long), ann))
    return out


def test_sequence_token_randomizer(samples, vocab):
    rnd = SimpleTokenRandomizer(vocab=vocab, p=.05)
    return [(rnd(s), a) for s, a in samples]


def test_masking_annotation(samples):
    masking = AnnotationMasking()
    return [(s, masking(torch.tensor(a, dtype=torch.float32))) for s, a in samples]


test_sequence_transform.__test__ = False
test_sequence_token_randomizer.__test__ = False
test_masking_annotation.__test__ = False


def test_data_processing(nb_annotations: int = NB_ANNOTATIONS) -> None:
    samples = create_random_samples(5, nb_annotations=nb_annotations)
    vocab = create_amino_acid_vocab()
    print("VOCAB:")
    print(vocab.get_itos())
    tr = test_sequence_transform(samples, vocab, 128)
    print("TRANSFORMED SEQUENCES:")
    for s, _ in tr:
        print(s, "\n")
    print("RANDOMIZED TOKEN SEQUENCES:")
    for s, _ in test_sequence_token_randomizer(tr, vocab):
        print(s, "\n")
    print("MASKED ANNOTATIONS:")
    for _, a in test_masking_annotation(samples):
        print(a, "\n")


test_data_processing.__test__ = False


def main(argv: Optional[List[str]] = None) -> dict:
    ap = argparse.ArgumentParser(description="ProteinBERT smoke pretraining (reference dummy_tests.py)")
    ap.add_argument("--iterations", type=int, default=250)
    ap.add_argument("--samples", type=int, default=100)
    ap.add_argument("--seq-len", type=int, default=256)
    ap.add_argument("--batch-size", type=int, default=BATCH_SIZE)
    ap.add_argument("--num-blocks", type=int, default=6)
    ap.add_argument("--annotations", type=int, default=NB_ANNOTATIONS)
    ap.add_argument("--save-path", default=".")
    ap.add_argument("--device", default=None)
    ap.add_argument("--backend", default="auto", choices=["auto", "hip", "torch"])
    ap.add_argument("--show-data", action="store_true", help="also run test_data_processing()")
    a = ap.parse_args(argv)
    logging.basicConfig(format="%(asctime)s [%(levelname)s]: %(message)s", level=logging.INFO)
    logging.info("Test pretraining initialization...")
    if a.show_data:
        test_data_processing(a.annotations)
    samples = create_random_samples(a.samples, 1, nb_annotations=a.annotations)
    df = pd.DataFrame(samples)
    print(df)
    dataset = UniRefGO_PretrainingDataset(df, seq_max_length=a.seq_len)
    loader = DataLoader(dataset=dataset, shuffle=True, num_workers=NUM_WORKERS, batch_size=a.batch_size,
                        collate_fn=collate_triples)
    device = torch.device(a.device or ("cuda" if torch.cuda.is_available() else "cpu"))
    model = ProteinBERT(sequences_length=a.seq_len, num_annotations=a.annotations, local_dim=128, global_dim=512,
                        key_dim=64, num_heads=4, num_blocks=a.num_blocks, device=device, backend=a.backend)
    print(f"\n {summary(model=model, col_names=['num_params', 'trainable'], col_width=20, row_settings=['var_names'])}\n")
    optimizer = torch.optim.Adam(params=model.parameters(), lr=2e-04)
    return pretrain(model=model, train_dataloader=loader, optimizer=optimizer,
                    local_loss_fn=CrossEntropyLoss(reduction="none"), global_loss_fn=BCELoss(reduction="none"),
                    max_batch_iterations=a.iterations, save_path=a.save_path, device=device)


if __name__ == "__main__":
    main()
