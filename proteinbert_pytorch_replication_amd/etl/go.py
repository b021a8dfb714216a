"""Gene Ontology OBO parsing (reference ``uniref_dataset.py:158-198, 323-360``).

``parse_go_annotations_meta(path)`` returns a DataFrame indexed by GO id with an integer ``index``
column, the OBO fields, ``direct_parents``/``direct_children`` (from ``is_a``) and the transitive
``all_ancestors``/``all_offspring`` closures (each term includes itself).
"""
from __future__ import annotations

import re
from typing import Dict, Iterable, Set

import numpy as np
import pandas as pd

ALL_FIELDS = ["id", "name", "namespace", "def", "is_a", "synonym", "alt_id", "subset", "is_obsolete", "xref",
              "relationship", "intersection_of", "disjoint_from", "consider", "comment", "replaced_by",
              "created_by", "creation_date", "property_value"]
LIST_FIELDS = {"synonym", "alt_id", "subset", "is_a", "xref", "relationship", "disjoint_from", "intersection_of",
               "consider", "property_value"}

_TERM = re.compile(r"\[Term\]\n((?:\w+: .*\n?)+)")
_FIELD = re.compile(r"(\w+): (.*)")


def parse_obo_terms(text: str):
    for m in _TERM.finditer(text):
        term = {f: [] for f in LIST_FIELDS}
        for line in m.group(1).splitlines():
            fm = _FIELD.match(line)
            if fm is None:
                continue
            field, value = fm.group(1), fm.group(2)
            if field not in ALL_FIELDS:
                raise ValueError(f"unknown OBO field {field!r}")
            if field in LIST_FIELDS:
                term[field].append(value)
            else:
                if field in term:
                    raise ValueError(f"duplicate OBO field {field!r} in {term.get('id')}")
                term[field] = value
        yield term


def parse_go_annotations_meta(meta_file_path: str) -> pd.DataFrame:
    with open(meta_file_path, "r") as f:
        terms = list(parse_obo_terms(f.read()))
    meta = pd.DataFrame(terms, columns=ALL_FIELDS)
    meta["is_obsolete"] = meta["is_obsolete"].fillna(False)
    if not meta["id"].is_unique:
        raise ValueError("GO ids are not unique")
    meta.set_index("id", drop=True, inplace=True)
    meta.insert(0, "index", np.arange(len(meta)))
    add_children_and_parents(meta)
    return meta


def add_children_and_parents(meta: pd.DataFrame) -> None:
    parents: Dict[str, Set[str]] = {go_id: set() for go_id in meta.index}
    children: Dict[str, Set[str]] = {go_id: set() for go_id in meta.index}
    names = meta["name"].to_dict()
    for go_id, is_a in meta["is_a"].items():
        for raw in is_a:
            parent_id, _, parent_name = raw.partition(" ! ")
            if parent_id not in parents:
                raise KeyError(f"{go_id}: unknown parent {parent_id}")
            if parent_name and names.get(parent_id) != parent_name:
                raise ValueError(f"{go_id}: parent name mismatch for {parent_id}")
            parents[go_id].add(parent_id)
            children[parent_id].add(go_id)
    meta["direct_parents"] = pd.Series(parents)
    meta["direct_children"] = pd.Series(children)
    roots = [g for g, p in parents.items() if not p]
    leaves = [g for g, c in children.items() if not c]
    meta["all_ancestors"] = pd.Series(index_to_all_ancestors(children, roots))
    meta["all_offspring"] = pd.Series(index_to_all_ancestors(parents, leaves))


def index_to_all_ancestors(index_to_direct_children: Dict[str, Iterable[str]], root_indices: Iterable[str]):
    """Level-wise propagation from the roots: every node's set = itself + all its ancestors."""
    out = {i: {i} for i in index_to_direct_children}
    frontier = set(root_indices)
    while frontier:
        nxt = set()
        for i in frontier:
            for child in index_to_direct_children[i]:
                out[child].update(out[i])
                nxt.add(child)
        frontier = nxt
    return out
