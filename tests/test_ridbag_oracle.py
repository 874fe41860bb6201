"""Embedded ridbag streams (oracle/ridbag_ref.py): encode/decode round trips and the header variants
the device decoder (orientdb_amd/csrc/ridbag.hip) must accept or refuse. CPU only."""
import random

import pytest

from oracle import ridbag_ref as R


@pytest.mark.parametrize("seed", range(10))
def test_round_trip(seed):
    rnd = random.Random(seed)
    rids = [(rnd.randrange(0, 40), rnd.randrange(0, 1 << 40)) for _ in range(rnd.randrange(0, 50))]
    uuid = bytes(rnd.randrange(256) for _ in range(16)) if seed % 2 else None
    s = R.encode_embedded(rids, uuid)
    assert len(s) == 1 + (16 if uuid else 0) + 4 + 10 * len(rids)  # ORidBag + OEmbeddedRidBag sizes
    assert R.decode(s) == rids


def test_layout_is_big_endian():
    s = R.encode_embedded([(11, 258)])
    assert s == bytes([1, 0, 0, 0, 1, 0, 11, 0, 0, 0, 0, 0, 0, 1, 2])


def test_refused_streams():
    with pytest.raises(ValueError):
        R.decode(R.encode_sbtree_pointer())
    with pytest.raises(ValueError):
        R.decode(R.encode_embedded([(1, 2), (3, 4)])[:-1])
    assert R.decode(b"") == []


def test_decoder_symbol_exported():
    import orientdb_amd._native as N
    assert N.lib().omx_ridbag_decode_csr is not None


# ---- SBTree-bonsai bags ------------------------------------------------------------------------------
def _bag(rnd, n, clusters=(11, 12, 13)):
    rids = sorted({(rnd.choice(clusters), rnd.randrange(0, 1 << 40)) for _ in range(n)})
    return [(r, rnd.choice((1, 1, 1, 2, 3))) for r in rids]


def _expand(counts):
    return [r for r, c in sorted(counts) for _ in range(c)]


@pytest.mark.parametrize("seed", range(8))
def test_sbtree_round_trip(seed):
    """Trees written bucket by bucket as OSBTreeBonsaiBucket.addEntry lays them out (random leaf sizes,
    buckets scattered over the pages, emptied leaves left in the sibling chain) and read back by the
    literal restatement of the reference iteration: the RIDs in RID order, each `count` times."""
    rnd = random.Random(seed)
    f = R.BonsaiFile(7, rng=random.Random(seed + 100))
    files = {7: f}
    for n in (1, 5, 109, 110, 500, 3000 if seed < 2 else 800):
        counts = _bag(rnd, n)
        root = f.build_tree(counts, rng=rnd, empty_leaf_every=(seed % 3) * 4)
        s = R.encode_sbtree_pointer(7, root[0], root[1], uuid=bytes(16) if seed % 2 else None)
        assert R.decode(s, files) == _expand(counts)


def test_sbtree_depth_and_layout():
    """A 20 000-entry bag: full leaves of 109 entries, 52-way internal nodes → three levels; page memory is
    little-endian except the RID position (big-endian, OLinkSerializer.java:76-89)."""
    rnd = random.Random(5)
    f = R.BonsaiFile(3)
    counts = _bag(rnd, 20000)
    root = f.build_tree(counts)
    b = R._Bucket({3: f}, 3, root)
    assert not b.leaf
    child = b.entry(0)[0]
    assert not R._Bucket({3: f}, 3, child).leaf
    assert R.decode(R.encode_sbtree_pointer(3, *root), {3: f}) == _expand(counts)
    leaf = R.BonsaiFile(4)
    p = leaf.alloc()
    leaf.write_bucket(p, True, [((11, 258), 2)])
    pg, o = leaf.pages[p[0]], p[1]
    pos = int.from_bytes(pg[o + R.O_POS:o + R.O_POS + 4], "little")
    assert pos == R.BUCKET_SIZE - 14
    assert bytes(pg[o + pos:o + pos + 14]) == bytes([11, 0, 0, 0, 0, 0, 0, 0, 1, 2, 2, 0, 0, 0])


def test_sbtree_changes_merge():
    """RIDBagIterator: tree entries and the serialized changes merged in RID order — a DiffChange adds to
    a tree counter or creates a RID, an AbsoluteChange sets it, a count <= 0 removes it."""
    f = R.BonsaiFile(9)
    counts = [((11, p), 1) for p in range(0, 40, 2)]
    root = f.build_tree(counts, leaf_fill=6)
    changes = [((11, 1), 0, 2),      # new RID, twice
               ((11, 4), 0, -1),     # removed
               ((11, 6), 1, 3),      # set to 3
               ((11, 7), 1, 0),      # absolute 0: not yielded
               ((11, 8), 0, 1),      # 1 + 1
               ((12, 0), 0, -2)]     # new RID with a negative count: not yielded
    got = R.decode(R.encode_sbtree_pointer(9, *root, changes=changes), {9: f})
    want = {}
    for r, c in counts:
        want[r] = c
    want[(11, 1)] = 2
    del want[(11, 4)]
    want[(11, 6)] = 3
    want[(11, 8)] = 2
    assert got == _expand(want.items())
    # a bag whose tree was never created (fileId -1): the changes alone
    s = R.encode_sbtree_pointer(-1, -1, -1, changes=[((11, 3), 0, 1), ((11, 5), 1, 2)])
    assert R.decode(s, {}) == [(11, 3), (11, 5), (11, 5)]


def test_sbtree_refused():
    f = R.BonsaiFile(9)
    root = f.build_tree([((11, 1), 1)])
    with pytest.raises(ValueError):  # the collection file is missing
        R.decode(R.encode_sbtree_pointer(8, *root), {9: f})
    with pytest.raises(ValueError):  # a root pointer past the file
        R.decode(R.encode_sbtree_pointer(9, 5, 0), {9: f})
    with pytest.raises(ValueError):  # truncated changes
        R.decode(R.encode_sbtree_pointer(9, *root, changes=[((11, 2), 0, 1)])[:-2], {9: f})
