"""Offline dataset construction: UniRef XML.gz + GO OBO -> SQLite -> pretraining dataset store.

Reference: ``ProteinBERT/uniref_dataset.py`` (E1-E5) and the two CLIs ``create_uniref_db.py`` and
``creare_uniref_h5_db.py`` (C1, C2).  CPU-only; not a performance target.  Implemented on the
standard library (``xml.etree.ElementTree`` streaming, ``sqlite3``) plus pandas, with a native
FASTA index reader instead of pyfaidx and the dataset written through
:class:`..data.store.ProteinStoreWriter` (HDF5 for ``*.h5`` paths, ``.pbxds`` otherwise).
"""
from .go import parse_go_annotations_meta, add_children_and_parents, index_to_all_ancestors  # noqa: F401
from .fasta import FastaIndex  # noqa: F401
from .uniref import UnirefToSqliteParser, etree_fast_iter  # noqa: F401
from .dataset import (create_h5_dataset, create_dataset_store, load_seqs_and_annotations,  # noqa: F401
                      encode_annotations_as_a_binary_matrix)
