"""Streaming UniRef XML.gz -> SQLite (reference ``uniref_dataset.py:25-155``, stage E1).

Semantics kept from the reference: one row per ``<entry>`` with ``tax_id`` (NaN when the
representative member has no NCBI taxonomy property), ``uniprot_name`` (the representative
member's dbReference id), ``go_annotations`` (JSON dict category -> GO ids), ``flat_go_annotations``,
``n_go_annotations``, ``complete_go_annotation_indices``, ``n_complete_go_annotations``; rows are
appended to table ``protein_annotations`` every ``chunk_size`` entries; per-GO ``count``/``freq``
columns are added to the meta frame after parsing.

Reference quirk (``uniref_dataset.py:124-126``): the "complete" (ancestor-closed) set is computed
and then discarded - the stored indices are the *direct* annotations, and ``filter(None, ...)``
also drops GO index 0.  ``reference_compat=True`` (default) reproduces that exactly so datasets
match the reference byte for byte; ``reference_compat=False`` stores the ancestor closure.

lxml is not importable in this image, so parsing uses ``xml.etree.ElementTree.iterparse`` with the
same fast-iter memory discipline (clear each finished entry and detach it from the root).
"""
from __future__ import annotations

import gzip
import json
import sqlite3
import xml.etree.ElementTree as ET
from collections import Counter
from typing import Callable, Dict, Iterable, List, Optional, Set

import numpy as np
import pandas as pd

from ..utils.log import log

NAMESPACE = "http://uniprot.org/uniref"
NS_PREFIX = "{%s}" % NAMESPACE
GO_ANNOTATION_CATEGORIES = ["GO Molecular Function", "GO Biological Process", "GO Cellular Component"]


def etree_fast_iter(path_or_file, tag: str, func: Callable, max_elements: Optional[int] = None) -> int:
    """Call ``func(i, 'end', elem)`` for each completed ``tag`` element, freeing it afterwards
    (reference ``_etree_fast_iter``, ``uniref_dataset.py:374-395``).  Returns the element count."""
    context = ET.iterparse(path_or_file, events=("start", "end"))
    root = None
    i = 0
    for event, elem in context:
        if root is None and event == "start":
            root = elem
            continue
        if event != "end" or elem.tag != tag:
            continue
        func(i, event, elem)
        elem.clear()
        if root is not None:
            # entries are direct children of the root: drop the processed ones
            for child in list(root):
                if child is elem:
                    root.remove(child)
                    break
        i += 1
        if max_elements is not None and i >= max_elements:
            break
    del context
    return i


class UnirefToSqliteParser:
    def __init__(self, uniref_xml_gz_file_path: str, go_annotations_meta: pd.DataFrame, sqlite_file_path: str,
                 verbose: bool = True, log_progress_every: int = 1000, chunk_size: int = 100000,
                 reference_compat: bool = True, max_entries: Optional[int] = None):
        self.uniref_xml_gz_file_path = uniref_xml_gz_file_path
        self.go_annotations_meta = go_annotations_meta
        self.sqlite_conn = sqlite3.connect(sqlite_file_path)
        self.verbose = verbose
        self.log_progress_every = log_progress_every
        self.chunk_size = chunk_size
        self.reference_compat = reference_compat
        self.max_entries = max_entries

        self.go_annotation_to_all_ancestors: Dict[str, Set[str]] = go_annotations_meta["all_ancestors"].to_dict()
        self.go_id_to_index: Dict[str, int] = go_annotations_meta["index"].to_dict()
        self.go_index_to_id = {int(v): k for k, v in self.go_id_to_index.items()}

        self.go_index_record_counter: Counter = Counter()
        self.unrecognized_go_annotations: Counter = Counter()
        self.n_records_with_any_go_annotation = 0
        self._chunk_indices: List[int] = []
        self._chunk_records: List[tuple] = []

    def _open(self):
        p = self.uniref_xml_gz_file_path
        return gzip.open(p, "rb") if p.endswith(".gz") else open(p, "rb")

    def parse(self) -> None:
        with self._open() as f:
            etree_fast_iter(f, NS_PREFIX + "entry", self._process_entry, self.max_entries)
        if self._chunk_records:
            self._save_current_chunk()
        if self.verbose:
            log("Ignored the following unrecognized GO annotations: %s" % self.unrecognized_go_annotations)
            log("Parsed %d records with any GO annotation." % self.n_records_with_any_go_annotation)
        counts = pd.Series({self.go_index_to_id[k]: v for k, v in self.go_index_record_counter.items()},
                           dtype=float)
        self.go_annotations_meta["count"] = counts.reindex(self.go_annotations_meta.index).fillna(0)
        denom = self.n_records_with_any_go_annotation
        self.go_annotations_meta["freq"] = self.go_annotations_meta["count"] / (denom if denom else np.nan)
        self.sqlite_conn.commit()
        if self.verbose:
            log("Done.")

    def close(self) -> None:
        self.sqlite_conn.close()

    # -- per entry ---------------------------------------------------------------------------
    def _process_entry(self, i: int, event: str, entry) -> None:
        if self.verbose and i % self.log_progress_every == 0:
            log(i, end="\r")
        reps = entry.findall(NS_PREFIX + "representativeMember")
        if len(reps) != 1:
            raise ValueError(f"entry {i}: expected one representativeMember, found {len(reps)}")
        refs = reps[0].findall(NS_PREFIX + "dbReference")
        if len(refs) != 1:
            raise ValueError(f"entry {i}: expected one dbReference, found {len(refs)}")
        db_ref = refs[0]
        protein_name = db_ref.attrib["id"]
        tax = [p for p in db_ref.findall(NS_PREFIX + "property") if p.attrib.get("type") == "NCBI taxonomy"]
        try:
            tax_id = int(tax[0].attrib["value"]) if len(tax) == 1 else np.nan
        except (KeyError, ValueError):
            tax_id = np.nan
        go = {cat: self._extract_go_category(entry, cat) for cat in GO_ANNOTATION_CATEGORIES}
        self._chunk_indices.append(i)
        self._chunk_records.append((tax_id, protein_name, go))
        if len(self._chunk_records) >= self.chunk_size:
            self._save_current_chunk()

    @staticmethod
    def _extract_go_category(entry, category: str) -> List[str]:
        return list({p.attrib["value"] for p in entry.findall(NS_PREFIX + "property")
                     if p.attrib.get("type") == category})

    def _get_go_annotation_all_ancestors(self, annotation: str) -> Set[str]:
        if annotation in self.go_annotation_to_all_ancestors:
            return self.go_annotation_to_all_ancestors[annotation]
        self.unrecognized_go_annotations[annotation] += 1
        return set()

    def _get_complete_go_annotations(self, go_annotations: Iterable[str]) -> Set[str]:
        return set().union(*[self._get_go_annotation_all_ancestors(a) for a in go_annotations])

    def _get_complete_go_annotation_indices(self, go_annotations: List[str]) -> List[int]:
        complete = self._get_complete_go_annotations(go_annotations)   # also counts unrecognized ids
        if self.reference_compat:
            return sorted(filter(None, map(self.go_id_to_index.get, go_annotations)))
        return sorted(self.go_id_to_index[a] for a in complete if a in self.go_id_to_index)

    def _save_current_chunk(self) -> None:
        df = pd.DataFrame(self._chunk_records, columns=["tax_id", "uniprot_name", "go_annotations"],
                          index=self._chunk_indices)
        df["flat_go_annotations"] = df["go_annotations"].apply(
            lambda d: sorted(set().union(*map(set, d.values()))))
        df["n_go_annotations"] = df["flat_go_annotations"].apply(len)
        df["complete_go_annotation_indices"] = df["flat_go_annotations"].apply(self._get_complete_go_annotation_indices)
        df["n_complete_go_annotations"] = df["complete_go_annotation_indices"].apply(len)
        self.n_records_with_any_go_annotation += int((df["n_complete_go_annotations"] > 0).sum())
        for idx in df["complete_go_annotation_indices"]:
            self.go_index_record_counter.update(idx)
        for col in ("go_annotations", "flat_go_annotations", "complete_go_annotation_indices"):
            df[col] = df[col].apply(json.dumps)
        df.to_sql("protein_annotations", self.sqlite_conn, if_exists="append")
        self._chunk_indices, self._chunk_records = [], []
