"""SQLite + FASTA -> pretraining dataset store (reference ``uniref_dataset.py:201-320, 363-371``, E3-E5).

``create_h5_dataset`` keeps the reference's two passes (count, then write in ``save_chunk_size``
chunks of a seeded shuffle) and its annotation vocabulary rule (GO ids with ``count >=
min_records_to_keep_annotation``, sorted).  The output goes through :class:`ProteinStoreWriter`:
the reference HDF5 layout for ``*.h5`` paths (h5py, or the dependency-free writer in
``data/hdf5.py``), the memory-mappable ``.pbxds`` directory otherwise (which the native loader reads).
"""
from __future__ import annotations

import json
import sqlite3
from typing import Dict, Iterable, Iterator, List, Optional, Sequence, Tuple

import numpy as np
import pandas as pd

from ..data.store import ProteinStoreWriter
from ..utils.iteration import to_chunks
from ..utils.log import log
from .fasta import FastaIndex


def load_seqs_and_annotations(protein_annotations_sqlite_db_file_path: str, fasta_file_path: str,
                              shuffle: bool = True, records_limit: Optional[int] = None, verbose: bool = True,
                              log_progress_every: int = 10000) -> Iterator[Tuple[str, str, List[int]]]:
    """Yield ``(uniprot_id, seq, go_annotation_indices)``; records whose ``UniRef90_<acc>`` is
    absent from the FASTA are skipped and counted (reference ``uniref_dataset.py:274-320``)."""
    if verbose:
        log("Loading %s records..." % ("all" if records_limit is None else records_limit))
    conn = sqlite3.connect(protein_annotations_sqlite_db_file_path)
    q = "SELECT uniprot_name, complete_go_annotation_indices FROM protein_annotations"
    if records_limit is not None:
        q += " LIMIT %d" % int(records_limit)
    df = pd.read_sql_query(q, conn)
    conn.close()
    if verbose:
        log("Loaded %d proteins and their GO annotations (%d columns: %s)" % (df.shape + (", ".join(df.columns),)))
    if shuffle:
        df = df.sample(frac=1, random_state=0)
    if verbose:
        log("Loading FASTA index (%s)..." % fasta_file_path)
    fa = FastaIndex(fasta_file_path)
    n_failed = 0
    try:
        for i, (uniprot_id, raw) in enumerate(zip(df["uniprot_name"], df["complete_go_annotation_indices"])):
            if verbose and i % log_progress_every == 0:
                log("%d/%d" % (i, len(df)), end="\r")
            fasta_id = "UniRef90_%s" % uniprot_id.split("_")[0]
            if fasta_id not in fa:
                n_failed += 1
                continue
            yield uniprot_id, fa.fetch(fasta_id), json.loads(raw)
    finally:
        fa.close()
    if verbose:
        log("Finished. Failed finding the sequence for %d of %d records." % (n_failed, len(df)))


def encode_annotations_as_a_binary_matrix(records_annotations: Sequence[Iterable[int]],
                                          annotation_to_index: Dict[int, int]) -> np.ndarray:
    masks = np.zeros((len(records_annotations), len(annotation_to_index)), dtype=bool)
    for i, anns in enumerate(records_annotations):
        for a in anns:
            j = annotation_to_index.get(a)
            if j is not None:
                masks[i, j] = True
    return masks


def _common_annotations(go_annotations_meta_csv_file_path: str, min_records_to_keep_annotation: int):
    meta = pd.read_csv(go_annotations_meta_csv_file_path, usecols=["id", "index", "count"], index_col=0)
    counts = meta["count"]
    common_ids = np.array(sorted(counts[counts >= min_records_to_keep_annotation].index))
    orig_to_common = {int(meta.loc[a, "index"]): i for i, a in enumerate(common_ids)}
    return common_ids, orig_to_common


def create_dataset_store(protein_annotations_sqlite_db_file_path: str, fasta_file_path: str,
                         go_annotations_meta_csv_file_path: str, output_path: str, shuffle: bool = True,
                         min_records_to_keep_annotation: int = 100, records_limit: Optional[int] = None,
                         save_chunk_size: int = 10000, verbose: bool = True, log_progress_every: int = 10000,
                         fmt: str = "auto") -> int:
    """Write the E3 store; returns the number of sequences written."""
    common_ids, orig_to_common = _common_annotations(go_annotations_meta_csv_file_path,
                                                     min_records_to_keep_annotation)
    if verbose:
        log("Will encode the %d most common annotations." % len(common_ids))
    if fmt == "auto":
        fmt = "h5" if output_path.endswith((".h5", ".hdf5")) else "pbxds"
    writer = ProteinStoreWriter(output_path, [str(a) for a in common_ids], fmt=fmt)
    it = load_seqs_and_annotations(protein_annotations_sqlite_db_file_path, fasta_file_path, shuffle=shuffle,
                                   records_limit=records_limit, verbose=verbose,
                                   log_progress_every=log_progress_every)
    for chunk in to_chunks(it, save_chunk_size):
        ids, seqs, anns = zip(*chunk)
        masks = encode_annotations_as_a_binary_matrix(anns, orig_to_common)
        for uid, seq, m in zip(ids, seqs, masks):
            writer.append_mask(uid, seq, m)
    n = len(writer)
    writer.close()
    if verbose:
        log("Wrote %d sequences to %s (%s). Done." % (n, output_path, fmt))
    return n


def create_h5_dataset(protein_annotations_sqlite_db_file_path: str, fasta_file_path: str,
                      go_annotations_meta_csv_file_path: str, output_h5_file_path: str, shuffle: bool = True,
                      min_records_to_keep_annotation: int = 100, records_limit: Optional[int] = None,
                      save_chunk_size: int = 10000, verbose: bool = True, log_progress_every: int = 10000) -> int:
    """Reference-named entry point (``uniref_dataset.py:201``): the reference HDF5 layout
    (``data/hdf5.py`` writes it when h5py is not importable)."""
    out = output_h5_file_path
    return create_dataset_store(protein_annotations_sqlite_db_file_path, fasta_file_path,
                                go_annotations_meta_csv_file_path, out, shuffle=shuffle,
                                min_records_to_keep_annotation=min_records_to_keep_annotation,
                                records_limit=records_limit, save_chunk_size=save_chunk_size, verbose=verbose,
                                log_progress_every=log_progress_every)
