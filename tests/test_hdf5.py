"""The dependency-free HDF5 reader/writer (``data/hdf5.py``) for the reference dataset layout.

The reference writes its pretraining dataset with h5py (``ProteinBERT/uniref_dataset.py:236-245``).
Neither h5py nor libhdf5 exists in this image and the reference ships no ``.h5`` fixture, so parity
with files written by the HDF5 library is unpinned: these tests round-trip our own files, check the
encoded structures field by field against the file-format specification, and feed the reader
hand-built variants (chunked + deflate + shuffle storage, version-2 object headers, continuation
blocks) that h5py produces with non-default options.
"""
import os
import struct
import zlib

import numpy as np
import pytest

from proteinbert_pytorch_replication_amd.data import hdf5 as h5
from proteinbert_pytorch_replication_amd.data.store import ProteinStore, ProteinStoreWriter, H5Store

AA = list("ACDEFGHIKLMNPQRSTVWY")


def _records(n, n_ann, seed=0):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        s = "".join(rng.choice(AA, int(rng.integers(0, 400))))
        out.append((f"UniRef90_P{i:05d}", s, rng.random(n_ann) < 0.05))
    return out


@pytest.fixture()
def h5file(tmp_path):
    ann = [f"GO:{i:07d}" for i in range(45)]
    recs = _records(3000, len(ann))
    p = str(tmp_path / "d.h5")
    assert h5.write_reference_h5(p, ann, recs) == len(recs)
    return p, ann, recs


def test_round_trip_values_shapes_dtypes(h5file):
    p, ann, recs = h5file
    assert sorted(os.listdir(os.path.dirname(p))) == ["d.h5"]          # side files removed
    with h5.H5File(p) as f:
        assert f.keys() == ["annotation_masks", "included_annotations", "seq_lengths", "seqs", "uniprot_ids"]
        assert f["seqs"].shape == (3000,) and f["seqs"].dtype == object
        assert f["seq_lengths"].dtype == np.int32
        assert f["annotation_masks"].shape == (3000, 45) and f["annotation_masks"].dtype == bool
        assert [a.decode() for a in f["included_annotations"][:]] == ann
        seqs, ids = f["seqs"][:], f["uniprot_ids"][:]
        masks, lens = f["annotation_masks"][:], f["seq_lengths"][:]
        for i, (uid, s, m) in enumerate(recs):
            assert seqs[i].decode() == s and ids[i].decode() == uid
            assert lens[i] == len(s)
            np.testing.assert_array_equal(masks[i], m)
        assert f["seqs"][-1].decode() == recs[-1][1]
        np.testing.assert_array_equal(f["annotation_masks"][10:20], np.stack([r[2] for r in recs[10:20]]))


def test_superblock_and_headers_follow_the_spec(h5file):
    p, _, _ = h5file
    raw = open(p, "rb").read()
    assert raw[:8] == b"\x89HDF\r\n\x1a\n"
    # v0 superblock: versions 0, 8-byte offsets/lengths, leaf K 4, internal K 16
    assert raw[8:16] == bytes([0, 0, 0, 0, 0, 8, 8, 0])
    assert struct.unpack_from("<HHI", raw, 16) == (4, 16, 0)
    base, fs, eof, drv = struct.unpack_from("<QQQQ", raw, 24)
    assert (base, fs, drv) == (0, h5.UNDEF, h5.UNDEF) and eof == len(raw)
    # root symbol-table entry: cache type 1, scratch = (B-tree, local heap)
    _, ohdr, cache, _, bt, heap = struct.unpack_from("<QQIIQQ", raw, 56)
    assert cache == 1 and raw[bt:bt + 4] == b"TREE" and raw[heap:heap + 4] == b"HEAP"
    # root object header v1 holds exactly one symbol-table message pointing at the same pair
    assert raw[ohdr] == 1 and struct.unpack_from("<H", raw, ohdr + 2)[0] == 1
    mt, ms = struct.unpack_from("<HH", raw, ohdr + 16)
    assert (mt, ms) == (0x11, 16) and struct.unpack_from("<QQ", raw, ohdr + 24) == (bt, heap)
    with h5.H5File(p) as f:
        # variable-length UTF-8 string over an unsigned char parent (h5py.string_dtype())
        t = f["seqs"].type
        assert (t.cls, t.vtype, t.cset, t.base.cls, t.base.size, t.base.signed) == (9, 1, 1, 0, 1, False)
        # numpy bool: enum over int8 {FALSE: 0, TRUE: 1}
        e = f["annotation_masks"].type
        assert e.cls == 8 and e.members == ["FALSE", "TRUE"] and e.values == [b"\x00", b"\x01"]
        assert e.base.size == 1 and e.base.signed
        lay = f["seqs"].layout
        assert lay["class"] == 1 and lay["size"] == 16 * 3000
        # global heap collections
        desc = np.frombuffer(raw, np.uint8, 16, lay["addr"])
        coll = int(desc[4:12].view("<u8")[0])
        assert raw[coll:coll + 5] == b"GCOL\x01" and struct.unpack_from("<Q", raw, coll + 8)[0] >= 4096


def test_empty_dataset_is_unallocated(tmp_path):
    p = str(tmp_path / "e.h5")
    h5.write_reference_h5(p, ["GO:1", "GO:2"], [])
    with h5.H5File(p) as f:
        assert f["seqs"].shape == (0,) and f["seqs"].layout["addr"] == h5.UNDEF
        assert f["annotation_masks"][:].shape == (0, 2)
        assert [a.decode() for a in f["included_annotations"][:]] == ["GO:1", "GO:2"]


def test_many_collections(tmp_path, monkeypatch):
    monkeypatch.setattr(h5._Collections, "TARGET", 8192)
    ann = ["GO:1"]
    recs = _records(400, 1, seed=3)
    p = str(tmp_path / "m.h5")
    h5.write_reference_h5(p, ann, recs)
    with h5.H5File(p) as f:
        seqs = f["seqs"][:]
        assert [s.decode() for s in seqs] == [r[1] for r in recs]
        assert len(f._heaps) > 10


# ------------------------------------------------------------------------------------------------
# hand-built variants the reader must accept
def _append(path, blob):
    with open(path, "r+b") as fh:
        fh.seek(0, 2)
        pos = fh.tell()
        pad = (-pos) % 8
        fh.write(b"\0" * pad + blob)
        end = fh.tell()
        fh.seek(40)
        fh.write(struct.pack("<Q", end))          # superblock end-of-file address
    return pos + pad


def _repoint(path, name, new_ohdr):
    """Point the root SNOD entry `name` at another object header."""
    f = h5.H5File(path)
    bt, heap = struct.unpack_from("<QQ", f.mm, 56 + 24)
    data = f._local_heap(heap)
    snod = struct.unpack_from("<Q", f.mm, bt + 24 + 8)[0]
    n = struct.unpack_from("<H", f.mm, snod + 6)[0]
    for i in range(n):
        e = snod + 8 + 40 * i
        if f._cstr(data + struct.unpack_from("<Q", f.mm, e)[0]) == name:
            f.close()
            with open(path, "r+b") as fh:
                fh.seek(e + 8)
                fh.write(struct.pack("<Q", new_ohdr))
            return
    raise KeyError(name)


def test_chunked_deflate_shuffle_dataset(h5file):
    p, _, recs = h5file
    lens = np.array([len(r[1]) for r in recs], np.int32)
    chunk = 512
    blobs, keys = [], []
    for c0 in range(0, len(lens), chunk):
        part = np.zeros(chunk, np.int32)
        part[:len(lens[c0:c0 + chunk])] = lens[c0:c0 + chunk]
        shuffled = part.view(np.uint8).reshape(-1, 4).T.copy().tobytes()   # byte planes
        blobs.append(zlib.compress(shuffled))
        keys.append(c0)
    addrs = []
    for b in blobs:
        addrs.append(_append(p, b))
    # one leaf node of the raw-data chunk B-tree (rank 1 -> 2 key dims incl. the element dim)
    node = b"TREE" + bytes([1, 0]) + struct.pack("<HQQ", len(blobs), h5.UNDEF, h5.UNDEF)
    for c0, a, b in zip(keys, addrs, blobs):
        node += struct.pack("<IIQQ", len(b), 0, c0, 0) + struct.pack("<Q", a)
    node += struct.pack("<IIQQ", 0, 0, len(lens), 0)
    tree = _append(p, node)
    msg = h5.H5Writer._msg
    space = struct.pack("<BBBB4x", 1, 1, 1, 0) + struct.pack("<QQ", len(lens), len(lens))
    layout = struct.pack("<BBBQII", 3, 2, 2, tree, chunk, 4)
    # filter pipeline v1: shuffle (2, client value = element size) then deflate (1, level 4)
    filt = struct.pack("<BB6x", 1, 2)
    filt += struct.pack("<HHHH", 2, 0, 0, 1) + struct.pack("<I", 4) + b"\0" * 4
    filt += struct.pack("<HHHH", 1, 0, 0, 1) + struct.pack("<I", 4) + b"\0" * 4
    hdr = h5.H5Writer._object_header(None, [msg(0x01, space), msg(0x03, h5._fixed_type(4, True)),
                                            msg(0x0B, filt), msg(0x08, layout)])
    _repoint(p, "seq_lengths", _append(p, hdr))
    with h5.H5File(p) as f:
        ds = f["seq_lengths"]
        assert ds.layout["class"] == 2 and [x[0] for x in ds.filters] == [2, 1]
        np.testing.assert_array_equal(ds[:], lens)
        np.testing.assert_array_equal(ds[700:1700], lens[700:1700])
        assert ds[2999] == lens[2999]


def test_version2_object_header_with_continuation(h5file):
    p, _, recs = h5file
    with h5.H5File(p) as f:
        msgs = f._messages(f._resolve("seqs"))
        bodies = [(mt, bytes(f.mm[q:q + ms])) for mt, q, ms in msgs]

    def v2(mt, body):
        return struct.pack("<BHB", mt, len(body), 0) + body

    # chunk 0: dataspace + datatype + a continuation message; the rest in an OCHK block
    head = [b for b in bodies if b[0] in (0x01, 0x03)]
    tail = [b for b in bodies if b[0] not in (0x01, 0x03)]
    cont_payload = b"OCHK" + b"".join(v2(mt, b) for mt, b in tail) + b"\0" * 4
    cont = _append(p, cont_payload)
    chunk0 = b"".join(v2(mt, b) for mt, b in head) + v2(0x10, struct.pack("<QQ", cont, len(cont_payload)))
    ohdr = b"OHDR" + bytes([2, 0x02]) + struct.pack("<I", len(chunk0)) + chunk0 + b"\0" * 4
    _repoint(p, "seqs", _append(p, ohdr))
    with h5.H5File(p) as f:
        seqs = f["seqs"][:]
        assert [s.decode() for s in seqs] == [r[1] for r in recs]


# ------------------------------------------------------------------------------------------------
# store / dataset integration
def test_store_writer_and_reader_h5(tmp_path):
    ann = [f"GO:{i}" for i in range(20)]
    recs = _records(200, len(ann), seed=5)
    p = str(tmp_path / "s.h5")
    w = ProteinStoreWriter(p, ann)
    assert w.fmt == "h5"
    for uid, s, m in recs[:100]:
        w.append_mask(uid, s, m)
    for uid, s, m in recs[100:]:
        w.append(uid, s, np.nonzero(m)[0])
    w.close()
    st = ProteinStore.open(p)
    assert isinstance(st, H5Store) and len(st) == 200 and st.included_annotations == ann
    for i in (0, 99, 100, 199):
        assert st.seq(i) == recs[i][1] and st.uniprot_id(i) == recs[i][0]
        np.testing.assert_array_equal(st.annotation_mask(i), recs[i][2])
    # same content as the .pbxds format
    q = str(tmp_path / "s.pbxds")
    w2 = ProteinStoreWriter(q, ann)
    for uid, s, m in recs:
        w2.append_mask(uid, s, m)
    w2.close()
    st2 = ProteinStore.open(q)
    for i in range(200):
        assert st2.seq(i) == st.seq(i)
        np.testing.assert_array_equal(st2.annotation_mask(i), st.annotation_mask(i))


def test_reference_dataset_class_reads_h5(tmp_path):
    from proteinbert_pytorch_replication_amd.data.datasets import UniRefGO_HDF5PretrainingDataset
    ann = [f"GO:{i}" for i in range(30)]
    recs = _records(64, len(ann), seed=7)
    p = str(tmp_path / "r.h5")
    h5.write_reference_h5(p, ann, recs)
    ds = UniRefGO_HDF5PretrainingDataset(p, seq_max_length=64, rank=1, world_size=2)
    assert len(ds) == 32
    X, Y, W = ds[0]
    assert X["local"].shape == (64,) and Y["global"].shape == (30,)
    np.testing.assert_array_equal(Y["global"].numpy() > 0, recs[1][2])


def test_user_block_files_are_refused_not_misread(h5file, tmp_path):
    """A file whose superblock sits behind a 512-byte user block resolves every address relative to
    the base address; the reader refuses it explicitly instead of reading wrong offsets."""
    p, _, _ = h5file
    q = str(tmp_path / "ub.h5")
    with open(p, "rb") as f, open(q, "wb") as g:
        g.write(b"\0" * 512 + f.read())
    with pytest.raises(NotImplementedError, match="user block"):
        h5.H5File(q)
