"""ETL CLIs with the reference flags (``create_uniref_db.py:20-72``, ``creare_uniref_h5_db.py:17-98``).

The reference scripts contain typos (``est=``/``ype=`` keyword arguments) that make argparse raise
at startup; these parsers keep the exact flag names, destinations, metavars and defaults, working.
"""
from __future__ import annotations

import argparse
from typing import List, Optional

from ..utils.cli_types import get_parser_file_type


def uniref_db_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="Create an sqlite DB from a raw UniRef file.")
    p.add_argument("--uniref-xml-gz-file", dest="uniref_xml_gz_file", metavar="/path/to/unirefXX.xml.gz",
                   type=get_parser_file_type(p, must_exist=True), required=True, help="Path to the raw UniRef file.")
    p.add_argument("--go-annotations-meta-file", dest="go_annotations_meta_file", metavar="/path/to/go.txt",
                   type=get_parser_file_type(p, must_exist=True), required=True,
                   help="Path to the specification file of all possible GO annotations (from CAFA).")
    p.add_argument("--output-sqlite-file", dest="output_sqlite_file", metavar="/path/to/uniref.db",
                   type=get_parser_file_type(p), required=True, help="Path to the save the output sqlite file.")
    p.add_argument("--output-go-annotations-meta-csv-file", dest="output_go_annotations_meta_csv_file",
                   metavar="/path/to/go_annotations.csv", type=get_parser_file_type(p), required=True,
                   help="Path to the save the output CSV file with metadata for all the GO annotations.")
    p.add_argument("--log-progress-every", dest="log_progress_every", metavar="1000", type=int, default=1000,
                   help="In verbose mode, log progress in increments of this many entries (default 1000).")
    p.add_argument("--chunk-size", dest="chunk_size", metavar="100000", type=int, default=100000,
                   help="The number of protein records per chunk written into the created DB.")
    p.add_argument("--silent", dest="silent", action="store_true", help="Run in silent mode.")
    p.add_argument("--complete-go-closure", dest="complete_go_closure", action="store_true",
                   help="Store the ancestor-closed GO index set (the reference stores the direct annotations).")
    p.add_argument("--max-entries", dest="max_entries", type=int, default=None,
                   help="Stop after this many UniRef entries (debugging).")
    return p


def run_uniref_db(args) -> None:
    from ..etl import UnirefToSqliteParser, parse_go_annotations_meta
    meta = parse_go_annotations_meta(args.go_annotations_meta_file)
    parser = UnirefToSqliteParser(args.uniref_xml_gz_file, meta, args.output_sqlite_file,
                                  verbose=not args.silent, log_progress_every=args.log_progress_every,
                                  chunk_size=args.chunk_size, reference_compat=not args.complete_go_closure,
                                  max_entries=args.max_entries)
    parser.parse()
    parser.close()
    meta.to_csv(args.output_go_annotations_meta_csv_file)


def uniref_h5_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="Create an h5 dataset from a UniRef sqlite DB.")
    p.add_argument("--protein-annotations-sqlite-db-file", dest="protein_annotations_sqlite_db_file",
                   metavar="/path/to/uniref.db", type=get_parser_file_type(p, must_exist=True), required=True,
                   help="The UniRef sqlite DB file.")
    p.add_argument("--protein-fasta-file", dest="protein_fasta_file", metavar="/path/to/uniref.fasta",
                   type=get_parser_file_type(p, must_exist=True), required=True,
                   help="The FASTA file with the full sequences of the proteins.")
    p.add_argument("--go-annotations-meta-csv-file", dest="go_annotations_meta_csv_file",
                   metavar="/path/to/go_annotations.csv", type=get_parser_file_type(p, must_exist=True),
                   required=True, help="Path to a CSV file with the count of each GO annotation.")
    p.add_argument("--output-h5-dataset-file", dest="output_h5_dataset_file", metavar="/path/to/dataset.h5",
                   type=get_parser_file_type(p), required=True,
                   help="Output dataset (HDF5 for *.h5 paths, else a .pbxds directory).")
    p.add_argument("--min-records-to-keep-annotation", dest="min_records_to_keep_annotation", metavar="100",
                   type=int, default=100, help="Minimal number of records required to encode an annotation.")
    p.add_argument("--log-progress-every", dest="log_progress_every", metavar="10000", type=int, default=10000,
                   help="In verbose mode, log progress in increments of this many records (default 10000).")
    p.add_argument("--records-limit", dest="records_limit", metavar="n", type=int, default=None,
                   help="Limit the number of loaded records. By default will load all records")
    p.add_argument("--save-chunk-size", dest="save_chunk_size", metavar="10000", type=int, default=10000,
                   help="The number of records to save per chunk.")
    p.add_argument("--no-shuffle", dest="no_shuffle", action="store_true", help="Disable the record shuffle.")
    p.add_argument("--silent", dest="silent", action="store_true", help="Run in silent mode.")
    p.add_argument("--format", dest="format", choices=["auto", "h5", "pbxds"], default="auto",
                   help="Output store format (auto: h5 for *.h5 paths, pbxds otherwise).")
    return p


def run_uniref_h5(args) -> None:
    from ..etl import create_dataset_store, create_h5_dataset
    kw = dict(shuffle=not args.no_shuffle, min_records_to_keep_annotation=args.min_records_to_keep_annotation,
              records_limit=args.records_limit, save_chunk_size=args.save_chunk_size, verbose=not args.silent,
              log_progress_every=args.log_progress_every)
    if args.format == "auto":
        create_h5_dataset(args.protein_annotations_sqlite_db_file, args.protein_fasta_file,
                          args.go_annotations_meta_csv_file, args.output_h5_dataset_file, **kw)
    else:
        create_dataset_store(args.protein_annotations_sqlite_db_file, args.protein_fasta_file,
                             args.go_annotations_meta_csv_file, args.output_h5_dataset_file, fmt=args.format, **kw)


def main_uniref_db(argv: Optional[List[str]] = None) -> None:
    run_uniref_db(uniref_db_parser().parse_args(argv))


def main_uniref_h5(argv: Optional[List[str]] = None) -> None:
    run_uniref_h5(uniref_h5_parser().parse_args(argv))
