"""ETL E1-E5 + CLIs C1/C2 on tiny synthetic UniRef/GO/FASTA fixtures (no reference fixtures exist)."""
import gzip
import json
import sqlite3

import numpy as np
import pandas as pd
import pytest

from proteinbert_pytorch_replication_amd.data.store import ProteinStore
from proteinbert_pytorch_replication_amd.etl import (FastaIndex, UnirefToSqliteParser,
                                                     encode_annotations_as_a_binary_matrix,
                                                     parse_go_annotations_meta)
from proteinbert_pytorch_replication_amd.cli.etl import main_uniref_db, main_uniref_h5

OBO = """format-version: 1.2

[Term]
id: GO:0000001
name: root
namespace: biological_process

[Term]
id: GO:0000002
name: child a
namespace: biological_process
is_a: GO:0000001 ! root

[Term]
id: GO:0000003
name: child b
namespace: biological_process
is_a: GO:0000001 ! root
synonym: "bee" EXACT []

[Term]
id: GO:0000004
name: grandchild
namespace: biological_process
is_a: GO:0000002 ! child a
is_a: GO:0000003 ! child b
is_obsolete: true

[Typedef]
id: part_of
name: part of
"""

NS = "http://uniprot.org/uniref"


def _entry(acc, tax, gos):
    props = "".join('<property type="%s" value="%s"/>' % (cat, g) for cat, g in gos)
    taxp = '<property type="NCBI taxonomy" value="%d"/>' % tax if tax is not None else ""
    return ('<entry id="UniRef90_%s"><name>x</name>%s<representativeMember>'
            '<dbReference type="UniProtKB ID" id="%s_HUMAN">%s</dbReference>'
            '<sequence length="3">MKV</sequence></representativeMember></entry>') % (acc, props, acc, taxp)


@pytest.fixture
def fixtures(tmp_path):
    obo = tmp_path / "go.txt"
    obo.write_text(OBO)
    entries = [
        _entry("P1", 9606, [("GO Molecular Function", "GO:0000002"), ("GO Biological Process", "GO:0000004")]),
        _entry("P2", None, [("GO Cellular Component", "GO:0000003"), ("GO Cellular Component", "GO:9999999")]),
        _entry("P3", 10090, []),
        _entry("P4", 7227, [("GO Molecular Function", "GO:0000001")]),
        _entry("P5", 7227, [("GO Biological Process", "GO:0000004")]),
    ]
    xml = '<?xml version="1.0"?><UniRef90 xmlns="%s" releaseDate="x">%s</UniRef90>' % (NS, "".join(entries))
    xml_gz = tmp_path / "uniref90.xml.gz"
    with gzip.open(xml_gz, "wb") as f:
        f.write(xml.encode())
    fasta = tmp_path / "uniref90.fasta"
    seqs = {"P1": "MKTAYIAKQRQISFVKSHFSRQ", "P2": "MSTNPKPQRKTKRNTNRRPQDVKFPGG" * 3, "P4": "ACDEFGHIK",
            "P5": "W" * 61}
    with open(fasta, "w") as f:
        for acc, s in seqs.items():
            f.write(">UniRef90_%s desc\n" % acc)
            for i in range(0, len(s), 10):
                f.write(s[i:i + 10] + "\n")
    return tmp_path, obo, xml_gz, fasta, seqs


def test_go_meta_closure(fixtures):
    _, obo, *_ = fixtures
    meta = parse_go_annotations_meta(str(obo))
    assert list(meta.index) == ["GO:0000001", "GO:0000002", "GO:0000003", "GO:0000004"]
    assert list(meta["index"]) == [0, 1, 2, 3]
    assert meta.loc["GO:0000004", "all_ancestors"] == {"GO:0000001", "GO:0000002", "GO:0000003", "GO:0000004"}
    assert meta.loc["GO:0000001", "all_offspring"] == {"GO:0000001", "GO:0000002", "GO:0000003", "GO:0000004"}
    assert meta.loc["GO:0000003", "synonym"] == ['"bee" EXACT []']
    assert meta.loc["GO:0000004", "is_obsolete"] == "true"
    assert meta.loc["GO:0000001", "is_obsolete"] is False
    assert meta.loc["GO:0000004", "direct_parents"] == {"GO:0000002", "GO:0000003"}


def test_fasta_index_matches_linear_parse(fixtures):
    _, _, _, fasta, seqs = fixtures
    fa = FastaIndex(str(fasta))
    for acc, s in seqs.items():
        assert fa.fetch("UniRef90_" + acc) == s
        assert fa.fetch("UniRef90_" + acc, 5, 14) == s[4:14]
    assert "UniRef90_P3" not in fa
    fa.close()
    fa2 = FastaIndex(str(fasta), build_index=False)  # reuses the written .fai
    assert fa2.index["UniRef90_P5"].rlen == 61


@pytest.mark.parametrize("compat", [True, False])
def test_uniref_to_sqlite(fixtures, compat):
    tmp, obo, xml_gz, *_ = fixtures
    meta = parse_go_annotations_meta(str(obo))
    db = tmp / ("u%d.db" % compat)
    p = UnirefToSqliteParser(str(xml_gz), meta, str(db), verbose=False, chunk_size=2, reference_compat=compat)
    p.parse()
    p.close()
    df = pd.read_sql_query("SELECT * FROM protein_annotations", sqlite3.connect(db))
    assert list(df["uniprot_name"]) == ["P1_HUMAN", "P2_HUMAN", "P3_HUMAN", "P4_HUMAN", "P5_HUMAN"]
    assert df["tax_id"].iloc[0] == 9606 and np.isnan(df["tax_id"].iloc[1])
    idx = [json.loads(x) for x in df["complete_go_annotation_indices"]]
    if compat:   # direct annotations only, and GO index 0 dropped by filter(None, ...)
        assert idx == [[1, 3], [2], [], [], [3]]
    else:
        assert idx == [[0, 1, 2, 3], [0, 2], [], [0], [0, 1, 2, 3]]
    assert p.unrecognized_go_annotations["GO:9999999"] == 1
    assert json.loads(df["flat_go_annotations"].iloc[0]) == ["GO:0000002", "GO:0000004"]
    assert "count" in meta and "freq" in meta
    assert meta.loc["GO:0000004", "count"] == (2 if compat else 2)


def test_binary_matrix():
    m = encode_annotations_as_a_binary_matrix([[5, 7], [], [9]], {5: 0, 9: 1})
    assert m.tolist() == [[True, False], [False, False], [False, True]]


def test_cli_end_to_end(fixtures):
    tmp, obo, xml_gz, fasta, seqs = fixtures
    db, csv, out = tmp / "u.db", tmp / "go.csv", tmp / "ds.pbxds"
    main_uniref_db(["--uniref-xml-gz-file", str(xml_gz), "--go-annotations-meta-file", str(obo),
                    "--output-sqlite-file", str(db), "--output-go-annotations-meta-csv-file", str(csv), "--silent",
                    "--complete-go-closure"])
    meta = pd.read_csv(csv, index_col=0)
    assert meta.loc["GO:0000001", "count"] == 4
    main_uniref_h5(["--protein-annotations-sqlite-db-file", str(db), "--protein-fasta-file", str(fasta),
                    "--go-annotations-meta-csv-file", str(csv), "--output-h5-dataset-file", str(out),
                    "--min-records-to-keep-annotation", "2", "--silent", "--format", "pbxds"])
    st = ProteinStore.open(str(out))
    assert st.included_annotations == ["GO:0000001", "GO:0000002", "GO:0000003", "GO:0000004"]
    assert len(st) == 4   # P3 has no sequence in the FASTA
    got = {st.uniprot_id(i): (st.seq(i), st.annotation_mask(i).tolist()) for i in range(len(st))}
    assert got["P1_HUMAN"] == (seqs["P1"], [True, True, True, True])
    assert got["P2_HUMAN"] == (seqs["P2"], [True, False, True, False])
    assert got["P4_HUMAN"] == (seqs["P4"], [True, False, False, False])
    # --no-shuffle keeps the sqlite order
    out2 = tmp / "ds2.pbxds"
    main_uniref_h5(["--protein-annotations-sqlite-db-file", str(db), "--protein-fasta-file", str(fasta),
                    "--go-annotations-meta-csv-file", str(csv), "--output-h5-dataset-file", str(out2),
                    "--min-records-to-keep-annotation", "3", "--silent", "--no-shuffle", "--records-limit", "2"])
    st2 = ProteinStore.open(str(out2) if out2.exists() else str(out2).rsplit(".", 1)[0] + ".pbxds")
    assert [st2.uniprot_id(i) for i in range(len(st2))] == ["P1_HUMAN", "P2_HUMAN"]
    assert st2.included_annotations == ["GO:0000001", "GO:0000002", "GO:0000003", "GO:0000004"][:1] + \
        [a for a in ["GO:0000002", "GO:0000003", "GO:0000004"] if meta.loc[a, "count"] >= 3]
    # the reference flags with an .h5 path write the reference HDF5 layout (no h5py needed)
    out3 = tmp / "ds3.h5"
    main_uniref_h5(["--protein-annotations-sqlite-db-file", str(db), "--protein-fasta-file", str(fasta),
                    "--go-annotations-meta-csv-file", str(csv), "--output-h5-dataset-file", str(out3),
                    "--min-records-to-keep-annotation", "2", "--silent", "--no-shuffle"])
    from proteinbert_pytorch_replication_amd.data.hdf5 import H5File
    with H5File(str(out3)) as f:
        assert f.keys() == ["annotation_masks", "included_annotations", "seq_lengths", "seqs", "uniprot_ids"]
        ids = [x.decode() for x in f["uniprot_ids"][:]]
        assert sorted(ids) == sorted(got)
        for i, uid in enumerate(ids):
            assert f["seqs"][i].decode() == got[uid][0] and f["seq_lengths"][i] == len(got[uid][0])
            assert f["annotation_masks"][i].tolist() == got[uid][1]
