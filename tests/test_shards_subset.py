"""CPU: IndexIVF::copy_subset_to and the IVF shard cloner on host lists.

copy_subset_to follows faiss/invlists/InvertedLists.cpp:91-175 (five subset
types); the cloner follows faiss/gpu/GpuCloner.cpp:283-317 (shard_type 1 = id
modulo, 2 = id range, 4 = list range).  The expected entries below are a
plain restatement of those loops over the same lists.  Indexes are read from
files written byte by byte (tests/test_io_format.py), so no device is used.
"""
import numpy as np
import pytest

from test_io_format import D, NLIST, ilar_bytes, ivf_prefix

SIZES = [5, 0, 3, 7, 1, 4, 9, 2]


def make_lists(seed=11):
    rng = np.random.default_rng(seed)
    sizes = SIZES[:NLIST]
    codes = [rng.random((n, D), dtype=np.float32) for n in sizes]
    ids = [rng.permutation(1000)[:n].astype(np.int64) for n in sizes]
    return sizes, codes, ids


def read_pair(amd, tmp_path, seed=11):
    sizes, codes, ids = make_lists(seed)
    fn = tmp_path / "src.index"
    fn.write_bytes(ivf_prefix(sum(sizes)) + ilar_bytes(sizes, codes, ids))
    src = amd.read_index(fn)
    dst = amd.read_index(fn)
    dst.reset()
    return src, dst, sizes, codes, ids


def expected(sizes, ids, st, a1, a2):
    """faiss/invlists/InvertedLists.cpp:91-175: (list, position) entries."""
    out = []
    ntotal = sum(sizes)
    accu_n = accu_a1 = accu_a2 = 0
    for l, n in enumerate(sizes):
        if st == 0:
            out += [(l, i) for i in range(n) if a1 <= ids[l][i] < a2]
        elif st == 1:
            out += [(l, i) for i in range(n) if ids[l][i] % a1 == a2]
        elif st == 2:
            nxt = accu_n + n
            n1, n2 = nxt * a1 // ntotal, nxt * a2 // ntotal
            out += [(l, i) for i in range(n1 - accu_a1, n2 - accu_a2)]
            accu_n, accu_a1, accu_a2 = nxt, n1, n2
        elif st == 3:
            out += [(l, i) for i in range(n * a2 // a1, n * (a2 + 1) // a1)]
        else:
            if a1 <= l < a2:
                out += [(l, i) for i in range(n)]
    return out


def check(idx, entries, codes, ids):
    per = {}
    for l, i in entries:
        per.setdefault(l, []).append(i)
    assert idx.ntotal == len(entries)
    for l in range(NLIST):
        want = per.get(l, [])
        assert idx.get_list_size(l) == len(want), l
        if want:
            assert np.array_equal(idx.list_ids(l), ids[l][want])
            got = idx.list_codes(l).view(np.float32).reshape(-1, D)
            assert np.array_equal(got, codes[l][want])


@pytest.mark.parametrize("st,a1,a2", [(0, 100, 600), (1, 3, 1), (2, 7, 19), (3, 3, 2),
                                      (4, 2, 5), (1, 1, 0), (2, 0, 20)])
def test_copy_subset_to(amd, tmp_path, st, a1, a2):
    src, dst, sizes, codes, ids = read_pair(amd, tmp_path)
    n = amd.copy_subset_to(src, dst, st, a1, a2)
    ent = expected(sizes, ids, st, a1, a2)
    assert n == len(ent)
    check(dst, ent, codes, ids)


@pytest.mark.parametrize("st,a1,a2", [(5, 0, 1), (2, 0, 21), (2, 5, 3), (3, 2, 2), (1, 0, 0)])
def test_copy_subset_rejects_bad_arguments(amd, tmp_path, st, a1, a2):
    src, dst, *_ = read_pair(amd, tmp_path)
    with pytest.raises(amd.FaissError):
        amd.copy_subset_to(src, dst, st, a1, a2)


@pytest.mark.parametrize("shard_type", [1, 2, 4])
@pytest.mark.parametrize("nshard", [2, 3])
def test_index_ivf_to_shards_partition(amd, tmp_path, shard_type, nshard):
    src, _, sizes, codes, ids = read_pair(amd, tmp_path, seed=5)
    sh = amd.index_ivf_to_shards(src, nshard, shard_type)
    assert sh.count() == nshard
    ntotal = sum(sizes)
    seen = []
    for i in range(nshard):
        part = sh.shard(i)
        if shard_type == 1:
            ent = expected(sizes, ids, 1, nshard, i)
        elif shard_type == 2:
            ent = expected(sizes, ids, 0, i * ntotal // nshard, (i + 1) * ntotal // nshard)
        else:
            ent = expected(sizes, ids, 4, i * NLIST // nshard, (i + 1) * NLIST // nshard)
        check(part, ent, codes, ids)
        seen += ent
    if shard_type != 2:  # id-range shards cover ids [0, ntotal) only
        assert sorted(seen) == sorted((l, i) for l in range(NLIST) for i in range(sizes[l]))
    assert sh.ntotal == len(seen)
