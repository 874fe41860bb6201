"""CPU restatement of the reference's embedded ridbag serialization.

TEST INFRASTRUCTURE ONLY: `tests/` may import this module as the checker / fixture writer; the product
path (orientdb_amd.ridbag, libomx omx_ridbag_decode_csr) never does.

Restates (C/ = core/src/main/java/com/orientechnologies/orient/core/):
  * C/db/record/ridbag/ORidBag.java:198-276 toStream — one config byte (bit 0: embedded delegate, bit 1:
    a 16-byte UUID follows), the UUID, then the delegate's serialization; :305-318 fromStream.
  * C/db/record/ridbag/embedded/OEmbeddedRidBag.java:424-460 serialize — int32 size, then every entry
    as a link; :462-472 deserialize / getSerializedSize :418-421 (size × RID_SIZE + INT_SIZE).
  * C/serialization/serializer/binary/impl/OLinkSerializer.java:47,54-58 — RID_SIZE = 2 + 8: short2bytes
    (cluster id), long2bytes (cluster position); OIntegerSerializer.java:53-58 — big-endian int32.

SBTree-bonsai bags (a bag of >= 40 entries by default, C/config/OGlobalConfiguration.java:356-358):
  * C/db/record/ridbag/sbtree/OSBTreeRidBag.java:818-880 serialize — after the config byte (bit 0
    clear) and the UUID: int64 fileId, int64 root pageIndex, int32 root pageOffset, int32 cached size
    (ignored since 1.7.5), then the changes: int32 count, count x (link, byte type, int32 value), all
    big-endian (serializeLiteral); :903-929 deserialize; ChangeSerializationHelper :197-249 (type 0 =
    DiffChange: counter + delta, type 1 = AbsoluteChange: the value; :118-195). The changes come from a
    ConcurrentSkipListMap (:60), so they are written in RID order.
  * the entries live in the collection file's pages (C/index/sbtreebonsai/local/): pages of
    DISK_CACHE_PAGE_SIZE = 64 KiB (OGlobalConfiguration.java:226-227) cut into buckets of
    SBTREEBONSAI_BUCKET_SIZE = 2 KiB (:338-340); a bucket pointer is (pageIndex, offset in the page)
    (OBonsaiBucketPointer.java). Page memory is native (little-endian) order (C/../common/directmemory/
    OByteBufferPool.java:150,329 ByteOrder.nativeOrder()). OSBTreeBonsaiBucket.java:44-60 offsets inside a
    bucket: free pointer 28, size 32, flags 36 (LEAF 1, DELETED 2), free-list pointer 37, left sibling 49,
    right sibling 61, tree size 73, key / value serializer ids 81 / 82, then the positions array (int32
    per entry, the entry's offset in the bucket) at 83. A leaf entry (:263-279 getEntry) is the key —
    OLinkSerializer native: int16 cluster id in native order, int64 position BIG-endian ("wrong
    implementation but needed for binary compatibility", OLinkSerializer.java:76-89) — then the int32
    value (the RID's multiplicity, native order). A non-leaf entry is (left child pointer, right child
    pointer, key), a pointer being int64 pageIndex + int32 pageOffset (OBonsaiBucketAbstract.java).
  * iteration (OSBTreeRidBag.java:256-425 RIDBagIterator, :427-514 SBTreeMapEntryIterator,
    :1066-1095): the tree's entries from firstKey() on (OSBTreeBonsaiLocal.java:848-935), in batches of
    1000 through loadEntriesMajor (:757-820: findBucket :1336-1374, then the leaves along their right
    siblings), merged in RID order with the changes; a tree entry with a change counts
    change.applyTo(value), a change-only RID applyTo(0); entries whose count is <= 0 are skipped; every
    RID is yielded `count` times.

No serialized bytes ship among the reference's test fixtures, so the format is pinned by these sources
(the round trips in tests/test_ridbag_oracle.py), not by golden vectors: parity unpinned.
"""
import struct

RID_SIZE = 10


def encode_embedded(rids, uuid=None):
    """ORidBag.toStream of an embedded bag holding `rids` (iterables of (cluster, position))."""
    cfg = 1 | (2 if uuid is not None else 0)
    out = bytearray([cfg])
    if uuid is not None:
        if len(uuid) != 16:
            raise ValueError("a UUID is 16 bytes")
        out += uuid
    rids = list(rids)
    out += struct.pack(">i", len(rids))
    for c, p in rids:
        out += struct.pack(">hq", c, p)
    return bytes(out)


def encode_sbtree_pointer(file_id=1, page=0, offset=0, changes=(), uuid=None, cached_size=0):
    """An SBTree delegate's stream (config bit 0 clear): OSBTreeRidBag.serialize :855-880. changes:
    ((cluster, position), type, value) with type 0 = DiffChange, 1 = AbsoluteChange, in RID order."""
    out = bytearray([2 if uuid is not None else 0])
    if uuid is not None:
        out += uuid
    out += struct.pack(">qqii", file_id, page, offset, cached_size)
    out += struct.pack(">i", len(changes))
    for (c, p), t, v in changes:
        out += struct.pack(">hqbi", c, p, t, v)
    return bytes(out)


# ---- SBTree-bonsai collection files ------------------------------------------------------------------
PAGE_SIZE = 64 * 1024
BUCKET_SIZE = 2 * 1024
O_FREE, O_SIZE, O_FLAGS, O_FREE_LIST, O_LEFT, O_RIGHT, O_TREE_SIZE, O_KEY_SER, O_VAL_SER, O_POS = (
    28, 32, 36, 37, 49, 61, 73, 81, 82, 83)
LEAF, DELETED = 1, 2
LINK_SERIALIZER_ID, INTEGER_SERIALIZER_ID = 9, 8
NULL_PTR = (-1, -1)
LEAF_ENTRY, NODE_ENTRY = 14, 34  # key + int32 value; two pointers + key


def _key_bytes(rid):
    return struct.pack("<h", rid[0]) + struct.pack(">q", rid[1])


def _key_of(b, o):
    return struct.unpack_from("<h", b, o)[0], struct.unpack_from(">q", b, o + 2)[0]


class BonsaiFile:
    """One collection file (collections_<cluster>.sbc): pages of PAGE_SIZE bytes, buckets of
    BUCKET_SIZE bytes allocated in the order `alloc` hands them out (a shuffled order spreads a tree's
    buckets over pages, as deletes and reuse do)."""

    def __init__(self, file_id, rng=None, page_size=PAGE_SIZE, bucket_size=BUCKET_SIZE):
        self.file_id, self.page_size, self.bucket_size = file_id, page_size, bucket_size
        self.pages = []
        self.free = []
        self.rng = rng

    def alloc(self):
        if not self.free:
            self.pages.append(bytearray(self.page_size))
            pi = len(self.pages) - 1
            slots = [(pi, off) for off in range(0, self.page_size, self.bucket_size)]
            if pi == 0:
                slots = slots[1:]  # page 0 offset 0 holds the sys bucket (OSysBucket)
            if self.rng is not None:
                self.rng.shuffle(slots)
            self.free = slots[::-1]
        return self.free.pop()

    def data(self):
        """The file's bytes as stored: its pages in order."""
        return b"".join(bytes(p) for p in self.pages)

    def _bucket(self, ptr):
        return self.pages[ptr[0]], ptr[1]

    def write_bucket(self, ptr, leaf, entries, left=NULL_PTR, right=NULL_PTR, tree_size=0):
        """OSBTreeBonsaiBucket(...) constructor + addEntry :355-413 for every entry in order: entries
        are laid out from the end of the bucket downwards, their offsets in the positions array."""
        pg, o = self._bucket(ptr)
        free = self.bucket_size
        for i, e in enumerate(entries):
            if leaf:
                (rid, value) = e
                data = _key_bytes(rid) + struct.pack("<i", value)
            else:
                (lc, rc, rid) = e
                data = struct.pack("<qi", *lc) + struct.pack("<qi", *rc) + _key_bytes(rid)
            free -= len(data)
            if free < O_POS + 4 * (i + 1):
                raise ValueError("bucket overflow")
            pg[o + free:o + free + len(data)] = data
            struct.pack_into("<i", pg, o + O_POS + 4 * i, free)
        struct.pack_into("<i", pg, o + O_FREE, free)
        struct.pack_into("<i", pg, o + O_SIZE, len(entries))
        pg[o + O_FLAGS] = LEAF if leaf else 0
        struct.pack_into("<qi", pg, o + O_FREE_LIST, *NULL_PTR)
        struct.pack_into("<qi", pg, o + O_LEFT, *left)
        struct.pack_into("<qi", pg, o + O_RIGHT, *right)
        struct.pack_into("<q", pg, o + O_TREE_SIZE, tree_size)
        pg[o + O_KEY_SER] = LINK_SERIALIZER_ID
        pg[o + O_VAL_SER] = INTEGER_SERIALIZER_ID

    # capacity of a bucket: positions-array slot + entry
    def leaf_capacity(self):
        return (self.bucket_size - O_POS) // (4 + LEAF_ENTRY)

    def node_capacity(self):
        return (self.bucket_size - O_POS) // (4 + NODE_ENTRY)

    def build_tree(self, counts, rng=None, empty_leaf_every=0, leaf_fill=None):
        """A B+-tree over sorted [(rid, count)] (count > 0): leaves of up to leaf_fill entries (random
        sizes with rng) linked by their siblings, internal levels of separators (child i < key <= child
        i + 1, findBucket :1369-1372) up to one root. Returns the root pointer."""
        items = sorted(counts)
        cap = self.leaf_capacity() if leaf_fill is None else min(leaf_fill, self.leaf_capacity())
        chunks, i = [], 0
        while i < len(items) or not chunks:
            n = cap if rng is None else rng.randint(1, cap)
            chunks.append(items[i:i + n])
            i += n
            if empty_leaf_every and len(chunks) % empty_leaf_every == 0:
                chunks.append([])  # a leaf emptied by removals: kept in the sibling chain
        ptrs = [self.alloc() for _ in chunks]
        for k, (p, ch) in enumerate(zip(ptrs, chunks)):
            self.write_bucket(p, True, ch, ptrs[k - 1] if k else NULL_PTR, ptrs[k + 1] if k + 1 < len(ptrs) else NULL_PTR,
                              tree_size=len(items) if len(ptrs) == 1 else 0)
        # first key at or after each child (separators); a trailing empty child gets a key past the last
        level = [(p, ch[0][0] if ch else None) for p, ch in zip(ptrs, chunks)]
        fanout = self.node_capacity() + 1
        while len(level) > 1:
            nxt_first = [None] * len(level)
            nxt = None
            for k in range(len(level) - 1, -1, -1):
                if level[k][1] is not None:
                    nxt = level[k][1]
                nxt_first[k] = nxt
            last = max((f for _, f in level if f is not None), default=(0, 0))
            sep = [nxt_first[k] if nxt_first[k] is not None else (last[0], last[1] + 1) for k in range(len(level))]
            groups, i = [], 0
            while i < len(level):
                n = fanout if rng is None else rng.randint(2, fanout)
                if len(level) - (i + n) == 1:
                    n += 1 if n < fanout else -1
                groups.append(list(range(i, min(i + n, len(level)))))
                i += n
            up = []
            for g in groups:
                p = self.alloc()
                entries = [(level[g[j]][0], level[g[j + 1]][0], sep[g[j + 1]]) for j in range(len(g) - 1)]
                if not entries:  # a lone child: nothing to separate, pass it up
                    up.append(level[g[0]])
                    continue
                self.write_bucket(p, False, entries, tree_size=len(items) if len(groups) == 1 else 0)
                up.append((p, level[g[0]][1] if level[g[0]][1] is not None else nxt_first[g[0]]))
            level = up
        return level[0][0]


class _Bucket:
    def __init__(self, files, file_id, ptr):
        f = files[file_id]
        if not (0 <= ptr[0] < len(f.pages)) or not (0 <= ptr[1] <= f.page_size - O_POS):
            raise ValueError("bucket pointer outside the collection file")
        self.b, self.o = f.pages[ptr[0]], ptr[1]
        self.leaf = (self.b[self.o + O_FLAGS] & LEAF) == LEAF

    def size(self):
        return struct.unpack_from("<i", self.b, self.o + O_SIZE)[0]

    def _pos(self, i):
        return self.o + struct.unpack_from("<i", self.b, self.o + O_POS + 4 * i)[0]

    def key(self, i):  # getKey :285-291
        return _key_of(self.b, self._pos(i) + (0 if self.leaf else 24))

    def entry(self, i):  # getEntry :263-279
        p = self._pos(i)
        if self.leaf:
            return _key_of(self.b, p), struct.unpack_from("<i", self.b, p + 10)[0]
        return struct.unpack_from("<qi", self.b, p), struct.unpack_from("<qi", self.b, p + 12), _key_of(self.b, p + 24)

    def find(self, key):  # find :187-204
        lo, hi = 0, self.size() - 1
        while lo <= hi:
            mid = (lo + hi) >> 1
            k = self.key(mid)
            if k < key:
                lo = mid + 1
            elif k > key:
                hi = mid - 1
            else:
                return mid
        return -(lo + 1)

    def right(self):
        return struct.unpack_from("<qi", self.b, self.o + O_RIGHT)


def tree_first_key(files, file_id, root):
    """OSBTreeBonsaiLocal.firstKey :848-935 (descends by the leftmost path, backtracking past empty
    buckets)."""
    path, ptr, idx = [], root, 0
    b = _Bucket(files, file_id, ptr)
    for _ in range(1 << 20):
        if b.leaf:
            if b.size() == 0:
                if not path:
                    return None
                ptr, idx = path.pop()
                idx += 1
            else:
                return b.key(0)
        else:
            if b.size() == 0 or idx > b.size():
                if not path:
                    return None
                ptr, idx = path.pop()
                idx += 1
            else:
                path.append((ptr, idx))
                ptr = b.entry(idx)[0] if idx < b.size() else b.entry(idx - 1)[1]
                idx = 0
        b = _Bucket(files, file_id, ptr)
    raise ValueError("SBTree descent did not end (a cycle of bucket pointers)")


def tree_entries_major(files, file_id, root, key, inclusive, limit):
    """loadEntriesMajor :757-820 with a listener that stops after `limit` entries."""
    ptr = root
    for _ in range(64):  # findBucket :1336-1374
        b = _Bucket(files, file_id, ptr)
        i = b.find(key)
        if b.leaf:
            break
        if i >= 0:
            e = b.entry(i)
        else:
            ins = -i - 1
            e = b.entry(ins - 1) if ins >= b.size() else b.entry(ins)
        ptr = e[1] if key >= e[2] else e[0]
    else:
        raise ValueError("SBTree deeper than 64 levels")
    out = []
    idx = (i if inclusive else i + 1) if i >= 0 else -i - 1
    for _ in range(1 << 24):
        for j in range(idx, b.size()):
            out.append(b.entry(j))
            if len(out) >= limit:
                return out
        ptr = b.right()
        if ptr[0] < 0:
            return out
        b = _Bucket(files, file_id, ptr)
        idx = 0
    raise ValueError("SBTree sibling chain did not end")


def tree_iterate(files, file_id, root, prefetch=1000):
    """SBTreeMapEntryIterator :427-514: (rid, value) of the whole tree in key order."""
    first = tree_first_key(files, file_id, root)
    if first is None:
        return []
    out = tree_entries_major(files, file_id, root, first, True, prefetch)
    batch = out
    while len(batch) == prefetch:
        batch = tree_entries_major(files, file_id, root, out[-1][0], False, prefetch)
        out += batch
    return out


def _apply(change, value):
    t, v = change
    return value + v if t == 0 else v  # DiffChange.applyTo / AbsoluteChange.applyTo


def iterate_sbtree_bag(files, file_id, root, changes):
    """RIDBagIterator :256-425 over (tree entries, changes) → the bag's RIDs in iteration order."""
    tree = tree_iterate(files, file_id, root) if file_id != -1 else []
    chg = dict((rid, (t, v)) for rid, t, v in changes)
    ti = iter([(k, _apply(chg[k], v) if k in chg else v) for k, v in tree])
    ti = (e for e in ti if e[1] > 0)  # nextChangedNotRemovedSBTreeEntry :1066-1095
    ci = ((rid, _apply((t, v), 0)) for rid, t, v in sorted(changes))
    ci = (e for e in ci if e[1] > 0)  # nextChangedNotRemovedEntry :410-424
    nt, nc = next(ti, None), next(ci, None)
    out = []
    while nt is not None or nc is not None:
        if nc is not None and nt is not None:
            if nc[0] < nt[0]:
                cur, nc = nc, next(ci, None)
            else:
                cur, nt = nt, next(ti, None)
                if nc is not None and nc[0] == cur[0]:
                    nc = next(ci, None)
        elif nc is not None:
            cur, nc = nc, next(ci, None)
        else:
            cur, nt = nt, next(ti, None)
        # next() returns the RID once before comparing its counter, so a tree counter <= 0 without a
        # change still yields it once (:305-309, hasNext :287-290)
        out += [cur[0]] * max(1, cur[1])
    return out


def decode(stream, files=None):
    """ORidBag.fromStream → the bag's RIDs in iteration order. SBTree bags need their collection files
    ({file id: BonsaiFile})."""
    if not stream:
        return []
    cfg = stream[0]
    if not cfg & 1:
        if files is None:
            raise ValueError("SBTree ridbag: entries are stored outside the record")
        o = 1 + (16 if cfg & 2 else 0)
        if o + 28 > len(stream):
            raise ValueError("truncated ridbag stream")
        fid, page, off, _size, n = struct.unpack_from(">qqiii", stream, o)
        o += 28
        if n < 0 or o + 15 * n > len(stream):
            raise ValueError("truncated ridbag stream")
        changes = []
        for i in range(n):
            c, p, t, v = struct.unpack_from(">hqbi", stream, o + 15 * i)
            if t not in (0, 1):
                raise ValueError("Change type is incorrect")
            changes.append(((c, p), t, v))
        if fid != -1 and fid not in files:
            raise ValueError("unknown collection file %d" % fid)
        return iterate_sbtree_bag(files, fid, (page, off), changes)
    o = 1 + (16 if cfg & 2 else 0)
    if o + 4 > len(stream):
        raise ValueError("truncated ridbag stream")
    (n,) = struct.unpack_from(">i", stream, o)
    o += 4
    if n < 0 or o + n * RID_SIZE > len(stream):
        raise ValueError("truncated ridbag stream")
    return [struct.unpack_from(">hq", stream, o + i * RID_SIZE) for i in range(n)]


def pack(c, p):
    return (c << 48) | p
