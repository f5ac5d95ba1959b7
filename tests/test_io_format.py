"""CPU: the library's reader on index files written here byte by byte from the
reference's format (faiss/impl/index_write.cpp:79-90, 243-297, 367-403,
631-638; OnDiskInvertedLists faiss/invlists/OnDiskInvertedLists.cpp:683-800),
in all three list storages: in-memory `ilar`, `ilar` mapped with
IO_FLAG_MMAP, and `ilod` lists in a separate data file.  No device is used:
reading fills the host mirrors only, and the lists are compared through the
C API getters.  Writing the read index back must give the same bytes."""
import struct

import numpy as np
import pytest

D, NLIST = 8, 6


def header(ntotal, d=D, metric=1):
    dummy = 1 << 20
    return struct.pack("<iqqqBi", d, ntotal, dummy, dummy, 1, metric)


def lists_data(seed=3):
    rng = np.random.default_rng(seed)
    sizes = [5, 0, 3, 7, 1, 4]
    codes = [rng.random((n, D), dtype=np.float32) for n in sizes]
    ids = [rng.integers(0, 1 << 40, n).astype(np.int64) for n in sizes]
    return sizes, codes, ids


def ivf_prefix(ntotal, nprobe=3, seed=4):
    cent = np.random.default_rng(seed).random((NLIST, D), dtype=np.float32)
    q = b"IxF2" + header(NLIST) + struct.pack("<Q", NLIST * D) + cent.tobytes()
    return (b"IwFl" + header(ntotal) + struct.pack("<QQ", NLIST, nprobe) + q +
            struct.pack("<bQ", 0, 0))


def ilar_bytes(sizes, codes, ids):
    cs = 4 * D
    b = b"ilar" + struct.pack("<QQ", NLIST, cs) + b"full" + struct.pack("<Q", NLIST)
    b += b"".join(struct.pack("<Q", n) for n in sizes)
    for n, c, i in zip(sizes, codes, ids):
        if n:
            b += c.tobytes() + i.tobytes()
    return b


def check_lists(idx, sizes, codes, ids):
    assert idx.ntotal == sum(sizes)
    for l in range(NLIST):
        assert idx.get_list_size(l) == sizes[l]
        assert np.array_equal(idx.list_ids(l), ids[l])
        assert np.array_equal(idx.list_codes(l).view(np.float32).reshape(-1, D),
                              codes[l].reshape(-1, D))


@pytest.mark.parametrize("flags", ["none", "mmap"])
def test_ilar_read_write_roundtrip(amd, tmp_path, flags):
    sizes, codes, ids = lists_data()
    raw = ivf_prefix(sum(sizes)) + ilar_bytes(sizes, codes, ids)
    fn = tmp_path / "a.index"
    fn.write_bytes(raw)
    idx = amd.read_index(fn, amd.IO_FLAG_MMAP if flags == "mmap" else 0)
    assert type(idx).__name__ == "IndexIVFFlat" and idx.nlist == NLIST and idx.nprobe == 3
    check_lists(idx, sizes, codes, ids)
    out = tmp_path / "b.index"
    amd.write_index(idx, out)
    assert out.read_bytes() == raw


def test_ilar_truncated_file_rejected(amd, tmp_path):
    sizes, codes, ids = lists_data()
    raw = ivf_prefix(sum(sizes)) + ilar_bytes(sizes, codes, ids)
    fn = tmp_path / "t.index"
    fn.write_bytes(raw[:-9])
    for fl in (0, amd.IO_FLAG_MMAP):
        with pytest.raises(amd.FaissError):
            amd.read_index(fn, fl)


def test_ilod_read_write_roundtrip(amd, tmp_path):
    sizes, codes, ids = lists_data(seed=5)
    cs = 4 * D
    data = tmp_path / "lists.ivfdata"
    blob, meta_lists = bytearray(), []
    for n, c, i in zip(sizes, codes, ids):
        cap = n + 2  # capacity slack: ids start after capacity codes
        off = len(blob)
        body = bytearray(cap * (cs + 8))
        body[:n * cs] = c.tobytes()
        body[cap * cs:cap * cs + 8 * n] = i.tobytes()
        blob += body
        meta_lists.append((n, cap, off))
    data.write_bytes(bytes(blob))
    name = str(data).encode()
    meta = b"ilod" + struct.pack("<QQQ", NLIST, cs, NLIST)
    meta += b"".join(struct.pack("<QQQ", *t) for t in meta_lists)
    meta += struct.pack("<Q", 0) + struct.pack("<Q", len(name)) + name
    meta += struct.pack("<Q", len(blob))
    raw = ivf_prefix(sum(sizes)) + meta
    fn = tmp_path / "o.index"
    fn.write_bytes(raw)
    idx = amd.read_index(fn)
    check_lists(idx, sizes, codes, ids)
    out = tmp_path / "p.index"
    amd.write_index(idx, out)
    assert out.read_bytes() == raw
    # a data file shorter than a list's extent is an error, not a fault
    data.write_bytes(bytes(blob[:len(blob) // 2]))
    with pytest.raises(amd.FaissError):
        amd.read_index(fn)


def test_mmap_index_resaved_in_place(amd, tmp_path):
    """write_index onto the very file the lists are mapped from (IO_FLAG_MMAP)
    must not truncate the mapping under the index: the file is written under
    a temporary name and renamed over the target."""
    sizes, codes, ids = lists_data(seed=6)
    raw = ivf_prefix(sum(sizes)) + ilar_bytes(sizes, codes, ids)
    fn = tmp_path / "m.index"
    fn.write_bytes(raw)
    idx = amd.read_index(fn, amd.IO_FLAG_MMAP)
    amd.write_index(idx, fn)
    assert fn.read_bytes() == raw
    check_lists(idx, sizes, codes, ids)  # still reads through the old mapping
    amd.write_index(idx, fn)
    assert fn.read_bytes() == raw
    assert sorted(p.name for p in tmp_path.iterdir()) == ["m.index"]  # no temporaries left


def test_write_keeps_symlink_and_mode(amd, tmp_path):
    """Only an existing regular file is replaced by rename, and it keeps its
    mode; a symlink stays a symlink (the file it names is replaced), and a
    FIFO is written in place."""
    import os
    import stat
    import threading
    sizes, codes, ids = lists_data(seed=8)
    raw = ivf_prefix(sum(sizes)) + ilar_bytes(sizes, codes, ids)
    src = tmp_path / "s.index"
    src.write_bytes(raw)
    idx = amd.read_index(src)
    real = tmp_path / "real.index"
    real.write_bytes(b"old")
    os.chmod(real, 0o640)
    link = tmp_path / "link.index"
    link.symlink_to(real)
    amd.write_index(idx, link)
    assert link.is_symlink() and real.read_bytes() == raw
    assert stat.S_IMODE(os.stat(real).st_mode) == 0o640
    fifo = tmp_path / "pipe"
    os.mkfifo(fifo)
    got = []
    t = threading.Thread(target=lambda: got.append(open(fifo, "rb").read()))
    t.start()
    amd.write_index(idx, fifo)
    t.join(30)
    assert got == [raw] and stat.S_ISFIFO(os.stat(fifo).st_mode)
    assert sorted(p.name for p in tmp_path.iterdir()) == [
        "link.index", "pipe", "real.index", "s.index"]


def test_ilod_data_file_rewritten_in_place(amd, tmp_path):
    """write_index_ondisk with the data file the lists are mapped from"""
    sizes, codes, ids = lists_data(seed=7)
    raw = ivf_prefix(sum(sizes)) + ilar_bytes(sizes, codes, ids)
    fn = tmp_path / "a.index"
    fn.write_bytes(raw)
    data = tmp_path / "lists.ivfdata"
    amd.write_index_ondisk(amd.read_index(fn), tmp_path / "o.index", data)
    idx = amd.read_index(tmp_path / "o.index")
    check_lists(idx, sizes, codes, ids)
    amd.write_index_ondisk(idx, tmp_path / "o.index", data)
    check_lists(idx, sizes, codes, ids)
    check_lists(amd.read_index(tmp_path / "o.index"), sizes, codes, ids)


def test_corrupt_list_extents_rejected(amd, tmp_path):
    """list sizes / capacities whose byte extent wraps around size_t"""
    sizes, codes, ids = lists_data(seed=8)
    cs = 4 * D
    # ilar mapped: a size of 2^61 (times cs + 8 = 40 wraps to a small number)
    bad = list(sizes)
    bad[2] = 1 << 61
    raw = ivf_prefix(sum(sizes)) + ilar_bytes(sizes, codes, ids)
    lo = raw.index(b"full") + 12
    raw = raw[:lo] + b"".join(struct.pack("<Q", n) for n in bad) + raw[lo + 8 * NLIST:]
    fn = tmp_path / "w.index"
    fn.write_bytes(raw)
    with pytest.raises(amd.FaissError):
        amd.read_index(fn, amd.IO_FLAG_MMAP)
    # ilod: capacity 2^61 with size 1
    data = tmp_path / "d.ivfdata"
    data.write_bytes(bytes(4 * (cs + 8)))
    name = str(data).encode()
    meta = b"ilod" + struct.pack("<QQQ", NLIST, cs, NLIST)
    meta += b"".join(struct.pack("<QQQ", *t) for t in
                     [(1, 1 << 61, 0)] + [(0, 0, 0)] * (NLIST - 1))
    meta += struct.pack("<Q", 0) + struct.pack("<Q", len(name)) + name
    meta += struct.pack("<Q", 4 * (cs + 8))
    fo = tmp_path / "w2.index"
    fo.write_bytes(ivf_prefix(1) + meta)
    with pytest.raises(amd.FaissError):
        amd.read_index(fo)
