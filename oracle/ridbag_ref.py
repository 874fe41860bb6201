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

No serialized bytes ship among the reference's test fixtures, so the format is pinned by these sources
(the round trip in tests/test_ridbag_oracle.py), not by golden vectors.
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


def encode_sbtree_pointer(file_id=1, page=0, offset=0):
    """An SBTree delegate's stream head (config bit 0 clear): what the device decoder must refuse."""
    return bytes([0]) + struct.pack(">qqi", file_id, page, offset) + struct.pack(">i", 0)


def decode(stream):
    """ORidBag.fromStream → the bag's RIDs in iteration order (embedded bags only)."""
    if not stream:
        return []
    cfg = stream[0]
    if not cfg & 1:
        raise ValueError("SBTree ridbag: entries are stored outside the record")
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
