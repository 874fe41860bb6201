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


# ---- SBTree-bonsai bags (omx_ridbag_decode_csr_ex) -----------------------------------------------------
def _mixed_streams(rp, col, f, rng, threshold=40, cluster=11):
    """Bags of >= threshold entries as SBTree bags in collection file f (RIDBag.toStream converts at
    RID_BAG_EMBEDDED_TO_SBTREEBONSAI_THRESHOLD, OGlobalConfiguration.java:356-358; the tree keeps one
    counter per distinct RID), the others embedded."""
    out, ntree = [], 0
    for v in range(len(rp) - 1):
        row = col[rp[v]:rp[v + 1]]
        if len(row) >= threshold:
            u, c = np.unique(row, return_counts=True)
            root = f.build_tree([((cluster, int(a)), int(b)) for a, b in zip(u, c)], rng=rng,
                                empty_leaf_every=7 if v % 5 == 0 else 0)
            out.append(R.encode_sbtree_pointer(f.file_id, *root, uuid=bytes(16) if v % 3 == 0 else None))
            ntree += 1
        else:
            out.append(R.encode_embedded([(cluster, int(w)) for w in row]))
    return out, ntree


@pytest.mark.parametrize("simple", [True, False], ids=["simple", "multigraph"])
def test_sbtree_and_embedded_rmat16_decode_to_the_csr(simple):
    """RMAT-16 (1 M entries): the hubs' bags as SBTree-bonsai trees (random leaf fill, buckets scattered
    over the pages, emptied leaves in the sibling chain; parallel edges as tree counters), the rest
    embedded: the device decodes the original CSR, every row in the bag's iteration order (RID order for
    a tree); a 2-hop MATCH on the decoded snapshot answers with the original's rows and digest."""
    import random

    import orientdb_amd as o
    from orientdb_amd.graph import rmat_csr
    from orientdb_amd.ridbag import decode_ridbags
    rp, col = rmat_csr(16, seed=3, simple=simple)
    V = len(rp) - 1
    f = R.BonsaiFile(5, rng=random.Random(1))
    streams, ntree = _mixed_streams(rp, col, f, random.Random(2))
    assert ntree > 1000
    vr = (np.uint64(11) << np.uint64(48)) | np.arange(V, dtype=np.uint64)
    grp, gcol = decode_ridbags(streams, vr, files={5: f.data()})
    assert np.array_equal(grp, rp.astype(np.uint64))
    assert np.array_equal(gcol, col)
    g0 = o.GraphSnapshot.person_knows(rp, col, seed=7)
    g1 = o.GraphSnapshot.person_knows(grp, gcol, seed=7)
    q = "MATCH {class:Person,as:a,where:(uid < 300)}-Knows->{as:b}-Knows->{as:c,where:(age < 20)} RETURN a, b, c"
    r0 = o.OMatchStatement(q).execute(g0, flags=o.OMX_FLAG_DIGEST)
    r1 = o.OMatchStatement(q).execute(g1, flags=o.OMX_FLAG_DIGEST)
    assert r0.info["n_rows"] == r1.info["n_rows"] > 0
    assert r0.info["digest"] == r1.info["digest"]


@pytest.mark.parametrize("seed", range(4))
def test_sbtree_bags_with_changes_match_the_oracle(seed):
    """Random bags against the literal restatement of OSBTreeRidBag's iterator (oracle/ridbag_ref.py):
    trees of 1 to 3000 entries with counters 1-3, serialized changes (DiffChange / AbsoluteChange, new,
    removed and re-counted RIDs), bags whose tree was never created (fileId -1), two collection files,
    RIDs over several clusters at scattered positions, regular edges (the bags hold edge records)."""
    import random

    from orientdb_amd.ridbag import decode_ridbags
    rnd = random.Random(seed)
    V = 400
    cl = [rnd.choice((11, 12)) for _ in range(V)]
    pos = rnd.sample(range(1 << 30), V)
    vrid = [(cl[v], pos[v]) for v in range(V)]
    vr = np.array([R.pack(*x) for x in vrid], np.uint64)
    files = {3: R.BonsaiFile(3, rng=random.Random(seed)), 9: R.BonsaiFile(9, rng=random.Random(seed + 1))}
    streams, want = [], []
    for v in range(V):
        kind = rnd.random()
        if kind < 0.3:
            row = [vrid[rnd.randrange(V)] for _ in range(rnd.randrange(0, 30))]
            streams.append(R.encode_embedded(row))
        else:
            n = rnd.choice((1, 5, 60, 300, 3000 if v % 50 == 0 else 200))
            keys = sorted({vrid[rnd.randrange(V)] for _ in range(n)})
            counts = [(k, rnd.choice((1, 1, 2, 3))) for k in keys]
            chg = {}
            for _ in range(rnd.randrange(0, 6) if kind < 0.7 else 0):
                k = keys[rnd.randrange(len(keys))] if rnd.random() < 0.6 else vrid[rnd.randrange(V)]
                chg[k] = (rnd.choice((0, 1)), rnd.randrange(-2, 4))
            changes = [(k, t, x) for k, (t, x) in sorted(chg.items())]
            if kind > 0.95:
                streams.append(R.encode_sbtree_pointer(-1, -1, -1, changes=changes))
            else:
                fid = rnd.choice((3, 9))
                root = files[fid].build_tree(counts, rng=rnd, empty_leaf_every=rnd.choice((0, 3)))
                streams.append(R.encode_sbtree_pointer(fid, *root, changes=changes,
                                                       uuid=bytes(range(16)) if v % 4 == 0 else None))
        row = R.decode(streams[-1], files)
        want.append([vrid.index(r) for r in row])
    grp, gcol = decode_ridbags(streams, vr, files={k: f.data() for k, f in files.items()})
    assert [gcol[grp[v]:grp[v + 1]].tolist() for v in range(V)] == want


@pytest.mark.parametrize("bad", ["missing_file", "root_past_file", "child_past_file", "changes_unsorted",
                                 "change_type", "no_files"])
def test_sbtree_refused(bad):
    import orientdb_amd as o
    from orientdb_amd.ridbag import decode_ridbags
    V = 64
    vr = np.array([R.pack(11, v) for v in range(V)], np.uint64)
    f = R.BonsaiFile(4)
    root = f.build_tree([((11, v), 1) for v in range(0, 64)], leaf_fill=5)
    stream = R.encode_sbtree_pointer(4, *root)
    files = {4: f.data()}
    if bad == "missing_file":
        files = {5: f.data()}
    elif bad == "root_past_file":
        stream = R.encode_sbtree_pointer(4, len(f.pages) + 2, 0)
    elif bad == "child_past_file":
        data = bytearray(f.data())
        b = R._Bucket({4: f}, 4, root)
        p = root[0] * R.PAGE_SIZE + root[1] + (b._pos(0) - root[1])
        data[p:p + 8] = (10 ** 6).to_bytes(8, "little")  # entry 0's left child page
        files = {4: bytes(data)}
    elif bad == "changes_unsorted":
        stream = R.encode_sbtree_pointer(4, *root, changes=[((11, 9), 0, 1), ((11, 2), 0, 1)])
    elif bad == "change_type":
        stream = R.encode_sbtree_pointer(4, *root, changes=[((11, 9), 7, 1)])
    streams = [stream] + [b""] * (V - 1)
    with pytest.raises(o.OmxError):
        decode_ridbags(streams, vr, files=None if bad == "no_files" else files)


@pytest.mark.parametrize("trees", [False, True], ids=["embedded", "sbtree"])
def test_edge_record_bags_to_edge_nodes(trees):
    """Bags of edge records decoded with their entries' RIDs (omx_ridbag_decode_edges) make an
    edge-records snapshot whose edge-node MATCH rows equal the record-level snapshot's. Each bag is written
    reversed (embedded: the decoded entry order differs from the original, so the RIDs must travel with
    their entries) or, from two entries on, as an SBTree (entries in RID order, k_runs_write's path)."""
    import random

    import orientdb_amd as o
    from orientdb_amd.graph import records_arrays
    from orientdb_amd.ridbag import decode_ridbags
    from tests.test_gpu_edges import edge_db
    db = edge_db(n=80, n_knows=400, n_likes=100, seed=9)
    V, classes, vclass, rids, sets, props, indexes, eprops = records_arrays(db, edge_records=True)
    f = R.BonsaiFile(7, rng=random.Random(2)) if trees else None
    new_sets, where = [], []
    base = 0
    orig = {}
    for es in sets:
        rp, col, er = es["out_rp"], es["out_col"], es["edge_rids"]
        for i, x in enumerate(er):
            orig[int(x)] = base + i
        base += len(er)
        streams = []
        for v in range(V):
            row = [(int(x) >> 48, int(x) & ((1 << 48) - 1)) for x in er[int(rp[v]):int(rp[v + 1])]]
            if trees and len(row) >= 2:
                root = f.build_tree([(r, 1) for r in sorted(row)], rng=random.Random(v))
                streams.append(R.encode_sbtree_pointer(f.file_id, *root))
            else:
                streams.append(R.encode_embedded(row[::-1]))
        files = {7: f.data()} if trees else None
        grp, gcol, ent = decode_ridbags(streams, rids, er, rids[col], files=files, entry_rids=True)
        assert len(ent) == len(er) and set(ent.tolist()) == set(er.tolist())
        if not trees:
            assert not np.array_equal(ent, er)  # the entries came back in another order
        new_sets.append({"cls": es["cls"], "out_rp": grp, "out_col": gcol, "edge_rids": ent})
        where += [orig[int(x)] for x in ent]
    idx = np.array(where, np.int64)
    eprops2 = [dict(p, values=np.asarray(p["values"])[idx], present=np.asarray(p["present"])[idx]) for p in eprops]
    g1 = o.GraphSnapshot.from_records(db, device=0, edge_records=True)
    g2 = o.GraphSnapshot(V, classes, vclass, rids, new_sets, props, indexes, 0, None, eprops2)
    for q in ("MATCH {class: Person, as: a}.outE('Knows'){as: e, where: (since > 2012)}.inV(){as: b} RETURN a, e, b",
              "MATCH {class: Person, as: b, where: (uid < 40)}.inE(){as: e}.outV(){as: a} RETURN $pathElements",
              "MATCH {class: Likes, as: e}.inV(){as: b, where: (age < 50)} RETURN e, b"):
        r1 = o.OMatchStatement(q).execute(g1, flags=o.OMX_FLAG_DIGEST)
        r2 = o.OMatchStatement(q).execute(g2, flags=o.OMX_FLAG_DIGEST)
        assert r1.info["n_rows"] == r2.info["n_rows"] > 0
        assert r1.info["digest"] == r2.info["digest"]
