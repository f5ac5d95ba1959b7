"""GPU: mmapped and on-disk inverted lists (§8(f) row 2).

* `read_index(fname, IO_FLAG_MMAP)` maps an `ilar` index file and streams the
  lists from the mapping into HBM (reference hook
  faiss/invlists/OnDiskInvertedLists.cpp:759-800, selected by
  faiss/impl/index_read.cpp:214-225) — the author's harness reads its index
  exactly this way (tutorial/cpp/benchmark-hnsw-ivf/benchmark_hnsw_ivf.cpp:361-362).
* `ilod` lists (OnDiskInvertedLists, :683-757): metadata in the index file,
  per list `codes[capacity*code_size]` then `ids[capacity]` at `offset` in a
  separate data file.  The hand-built file below restates that layout
  independently of the library (capacity slack, out-of-order offsets, a free
  slot table), so the reader is checked against the reference's format, not
  against our own writer.
"""
import struct

import numpy as np
import pytest

from conftest import assert_same_results, rand

pytestmark = pytest.mark.gpu

DESCS = ["IVF32,Flat", "IVF32,PQ8"]


def build(amd, orc, desc, d=32, nb=5000, seed=81):
    xb = rand(orc, nb, d, seed)
    idx = amd.index_factory(d, desc)
    idx.train(xb)
    idx.add(xb)
    idx.nprobe = 6
    return idx, xb


@pytest.mark.parametrize("desc", DESCS)
def test_mmap_read_same_results_and_bytes(amd, orc, gpu, tmp_path, desc):
    idx, xb = build(amd, orc, desc)
    xq = rand(orc, 200, 32, 82)
    D, I = idx.search(xq, 10)
    fn = tmp_path / "a.index"
    amd.write_index(idx, fn)
    idx2 = amd.read_index(fn, amd.IO_FLAG_MMAP)
    idx2.nprobe = 6
    assert idx2.ntotal == idx.ntotal
    D2, I2 = idx2.search(xq, 10)
    assert_same_results(D2, I2, D, I)
    for l in (0, 7, 31):
        assert np.array_equal(idx2.list_ids(l), idx.list_ids(l))
        assert np.array_equal(idx2.list_codes(l), idx.list_codes(l))
    fn2 = tmp_path / "b.index"
    amd.write_index(idx2, fn2)
    assert fn.read_bytes() == fn2.read_bytes()


@pytest.mark.parametrize("desc", DESCS)
def test_add_after_mmap_read(amd, orc, gpu, tmp_path, desc):
    # the mapped lists are copied to host memory before the append
    idx, xb = build(amd, orc, desc)
    fn = tmp_path / "a.index"
    amd.write_index(idx, fn)
    idx2 = amd.read_index(fn, amd.IO_FLAG_MMAP)
    extra = rand(orc, 700, 32, 83)
    idx.add(extra)
    idx2.add(extra)
    idx.nprobe = idx2.nprobe = 6
    xq = rand(orc, 150, 32, 84)
    D, I = idx.search(xq, 10)
    D2, I2 = idx2.search(xq, 10)
    assert_same_results(D2, I2, D, I)


def test_mmap_unknown_hook_rejected(amd, orc, gpu, tmp_path):
    idx, _ = build(amd, orc, "IVF32,Flat")
    fn = tmp_path / "a.index"
    amd.write_index(idx, fn)
    with pytest.raises(amd.FaissError):
        amd.read_index(fn, amd.IO_FLAG_SKIP_IVF_DATA | 0x12340000)


@pytest.mark.parametrize("desc", DESCS)
def test_write_index_ondisk_roundtrip(amd, orc, gpu, tmp_path, desc):
    idx, xb = build(amd, orc, desc)
    xq = rand(orc, 200, 32, 85)
    D, I = idx.search(xq, 10)
    fn, data = tmp_path / "o.index", tmp_path / "o.ivfdata"
    amd.write_index_ondisk(idx, fn, data)
    cs = idx.code_size
    assert data.stat().st_size == idx.ntotal * (cs + 8)
    idx2 = amd.read_index(fn)
    idx2.nprobe = 6
    D2, I2 = idx2.search(xq, 10)
    assert_same_results(D2, I2, D, I)
    # write_index of an ilod-backed index keeps pointing at the data file
    fn2 = tmp_path / "p.index"
    amd.write_index(idx2, fn2)
    assert fn2.read_bytes() == fn.read_bytes()


def test_ondisk_same_dir(amd, orc, gpu, tmp_path):
    idx, xb = build(amd, orc, "IVF32,Flat")
    xq = rand(orc, 100, 32, 86)
    D, I = idx.search(xq, 10)
    a, b = tmp_path / "a", tmp_path / "b"
    a.mkdir()
    b.mkdir()
    amd.write_index_ondisk(idx, a / "x.index", a / "x.ivfdata")
    (b / "x.index").write_bytes((a / "x.index").read_bytes())
    (b / "x.ivfdata").write_bytes((a / "x.ivfdata").read_bytes())
    (a / "x.ivfdata").unlink()
    with pytest.raises(amd.FaissError):
        amd.read_index(b / "x.index")  # stored path is a/x.ivfdata
    idx2 = amd.read_index(b / "x.index", amd.IO_FLAG_ONDISK_SAME_DIR)
    idx2.nprobe = 6
    D2, I2 = idx2.search(xq, 10)
    assert_same_results(D2, I2, D, I)


def _ilod_tail_len(nlist, nslots, fname):
    # "ilod", nlist, code_size, vector<List> (24 B each), vector<Slot> (16 B),
    # vector<char> filename, totsize  (OnDiskInvertedLists.cpp:683-704)
    return 4 + 8 + 8 + (8 + 24 * nlist) + (8 + 16 * nslots) + (8 + len(fname)) + 8


@pytest.mark.parametrize("desc", DESCS)
def test_handbuilt_ilod_with_capacity_slack(amd, orc, gpu, tmp_path, desc):
    idx, xb = build(amd, orc, desc)
    nlist, cs = 32, idx.code_size
    xq = rand(orc, 200, 32, 87)
    D, I = idx.search(xq, 10)
    fn, data = tmp_path / "o.index", tmp_path / "o.ivfdata"
    amd.write_index_ondisk(idx, fn, data)
    raw = fn.read_bytes()
    prefix = raw[:len(raw) - _ilod_tail_len(nlist, 0, str(data).encode())]
    assert raw[len(prefix):len(prefix) + 4] == b"ilod"
    # new data file: lists in reverse order, capacity = size + 3, 64-B gaps
    blob, lists, slots = bytearray(), [], []
    for l in reversed(range(nlist)):
        ids = idx.list_ids(l)
        codes = idx.list_codes(l)
        n = len(ids)
        cap = n + 3
        blob += b"\xee" * 64
        slots.append((len(blob) - 64, 64))
        off = len(blob)
        body = bytearray(b"\xcd" * (cap * (cs + 8)))
        body[:n * cs] = codes.tobytes()
        body[cap * cs:cap * cs + 8 * n] = ids.astype("<i8").tobytes()
        blob += body
        lists.append((l, n, cap, off))
    lists.sort()
    data2 = tmp_path / "slack.ivfdata"
    data2.write_bytes(bytes(blob))
    name = str(data2).encode()
    meta = b"ilod" + struct.pack("<QQ", nlist, cs)
    meta += struct.pack("<Q", nlist) + b"".join(struct.pack("<QQQ", n, c, o) for _, n, c, o in lists)
    meta += struct.pack("<Q", len(slots)) + b"".join(struct.pack("<QQ", o, c) for o, c in slots)
    meta += struct.pack("<Q", len(name)) + name + struct.pack("<Q", len(blob))
    fn2 = tmp_path / "slack.index"
    fn2.write_bytes(prefix + meta)
    idx2 = amd.read_index(fn2)
    idx2.nprobe = 6
    for l in range(nlist):
        assert np.array_equal(idx2.list_ids(l), idx.list_ids(l))
        assert np.array_equal(idx2.list_codes(l), idx.list_codes(l))
    D2, I2 = idx2.search(xq, 10)
    assert_same_results(D2, I2, D, I)
