"""Ridbag ingest on the device (omx_ridbag_decode_csr, orientdb_amd/csrc/ridbag.hip) against the
restated stream format (oracle/ridbag_ref.py: ORidBag.toStream / OEmbeddedRidBag.serialize). The streams
are written by the oracle's encoder from known CSRs; the decoded CSR must equal them entry for entry."""
import numpy as np
import pytest

from oracle import ridbag_ref as R

pytestmark = pytest.mark.gpu


def _streams(rp, col, rid_of, uuid_every=0, rng=None):
    out = []
    for v in range(len(rp) - 1):
        row = [int(x) for x in col[rp[v]:rp[v + 1]]]
        if not row and v % 3 == 0:
            out.append(b"")  # the vertex has no out_ field at all
            continue
        uuid = bytes(rng.integers(0, 256, 16, dtype=np.uint8)) if uuid_every and v % uuid_every == 0 else None
        out.append(R.encode_embedded([rid_of(w) for w in row], uuid))
    return out


@pytest.fixture(scope="module")
def csr10():
    from orientdb_amd.graph import rmat_csr
    return rmat_csr(10, simple=False, seed=5)


def test_lightweight_canonical(csr10):
    from orientdb_amd.ridbag import decode_ridbags
    rp, col = csr10
    V = len(rp) - 1
    rng = np.random.default_rng(0)
    streams = _streams(rp, col, lambda w: (11, w), uuid_every=7, rng=rng)
    vr = np.array([R.pack(11, v) for v in range(V)], np.uint64)
    grp, gcol = decode_ridbags(streams, vr)
    assert np.array_equal(grp, rp.astype(np.uint64))
    assert np.array_equal(gcol, col)


def test_arbitrary_rids_and_edge_records(csr10):
    from orientdb_amd.ridbag import decode_ridbags
    rp, col = csr10
    V, E = len(rp) - 1, len(col)
    rng = np.random.default_rng(1)
    # vertices spread over clusters 11..14 at random positions (not the canonical one-cluster layout)
    cl = rng.integers(11, 15, V)
    pos = rng.permutation(1 << 20)[:V]
    vr = np.array([R.pack(int(c), int(p)) for c, p in zip(cl, pos)], np.uint64)
    streams = _streams(rp, col, lambda w: (int(cl[w]), int(pos[w])))
    grp, gcol = decode_ridbags(streams, vr)
    assert np.array_equal(gcol, col)
    # regular edges: the out_ bags hold edge records #20:k whose `in` field is the neighbour
    eorder = rng.permutation(E)  # edge record #20:epos[i] is CSR entry i
    epos = np.empty(E, np.int64)
    epos[eorder] = np.arange(E)
    streams = [R.encode_embedded([(20, int(epos[i])) for i in range(int(rp[v]), int(rp[v + 1]))]) for v in range(V)]
    erids = np.array([R.pack(20, int(epos[i])) for i in range(E)], np.uint64)
    etargets = vr[col]
    grp, gcol = decode_ridbags(streams, vr, erids, etargets)
    assert np.array_equal(grp, rp.astype(np.uint64))
    assert np.array_equal(gcol, col)


@pytest.mark.parametrize("bad", ["sbtree", "truncated", "unknown_rid", "unknown_edge"])
def test_refused_streams(csr10, bad):
    import orientdb_amd as o
    from orientdb_amd.ridbag import decode_ridbags
    rp, col = csr10
    V = len(rp) - 1
    vr = np.array([R.pack(11, v) for v in range(V)], np.uint64)
    streams = _streams(rp, col, lambda w: (11, w))
    er = et = None
    if bad == "sbtree":
        streams[5] = R.encode_sbtree_pointer()
    elif bad == "truncated":
        streams[7] = R.encode_embedded([(11, 1), (11, 2)])[:-3]
    elif bad == "unknown_rid":
        streams[9] = R.encode_embedded([(11, 1), (11, V + 5)])
    else:
        streams = [R.encode_embedded([(20, 0), (20, 1)])] + [b""] * (V - 1)
        er = np.array([R.pack(20, 0)], np.uint64)
        et = np.array([R.pack(11, 3)], np.uint64)
    with pytest.raises(o.OmxError):
        decode_ridbags(streams, vr, er, et)


def test_ingested_snapshot_answers_like_the_original():
    """RMAT-16: bags written from the CSR, decoded on the device, snapshotted, queried: the same rows."""
    import orientdb_amd as o
    from orientdb_amd.graph import rmat_csr
    from orientdb_amd.ridbag import decode_ridbag_blob
    rp, col = rmat_csr(16, seed=3)
    V = len(rp) - 1
    # the streams built vectorised: [cfg=1][count BE][(11 BE16, v BE64)...] per vertex
    deg = np.diff(rp.astype(np.int64))
    sizes = 5 + 10 * deg
    offs = np.zeros(V + 1, np.uint64)
    offs[1:] = np.cumsum(sizes)
    blob = np.zeros(int(offs[-1]), np.uint8)
    starts = offs[:-1].astype(np.int64)
    blob[starts] = 1
    cnt = deg.astype(">u4").view(np.uint8).reshape(V, 4)
    for k in range(4):
        blob[starts + 1 + k] = cnt[:, k]
    entry_base = np.repeat(starts + 5, deg) + 10 * (np.arange(len(col)) - np.repeat(rp[:-1].astype(np.int64), deg))
    ent = np.zeros((len(col), 10), np.uint8)
    ent[:, 1] = 11
    ent[:, 2:] = col.astype(">u8").view(np.uint8).reshape(-1, 8)
    for k in range(10):
        blob[entry_base + k] = ent[:, k]
    vr = (np.uint64(11) << np.uint64(48)) | np.arange(V, dtype=np.uint64)
    grp, gcol = decode_ridbag_blob(blob.tobytes(), offs, vr)
    assert np.array_equal(gcol, col)
    g0 = o.GraphSnapshot.person_knows(rp, col, seed=7)
    g1 = o.GraphSnapshot.person_knows(grp, gcol, seed=7)
    q = "MATCH {class:Person,as:a,where:(uid < 300)}-Knows->{as:b}-Knows->{as:c,where:(age < 20)} RETURN a, b, c"
    r0 = o.OMatchStatement(q).execute(g0, flags=o.OMX_FLAG_DIGEST)
    r1 = o.OMatchStatement(q).execute(g1, flags=o.OMX_FLAG_DIGEST)
    assert r0.info["n_rows"] == r1.info["n_rows"] > 0
    assert r0.info["digest"] == r1.info["digest"]
