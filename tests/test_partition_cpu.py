"""The 1-D partitioned path on CPU.

* the partition generator (omx_rmat_generate_part) yields exactly the rows of the full RMAT graph and of
  its transpose for the vertices a rank owns;
* partitioned snapshots load host-only, explain like the full one, and reject inconsistent ranges;
* two gloo ranks run a numpy restatement of the executor's exchange (exec.hip route_owner /
  route_hash: rows travel to owner(row[src]) before every hop, and by tuple hash before a distinct
  projection) over their own partitions; the union of their rows equals the oracle DFS on the full
  graph, and the hash exchange leaves every distinct tuple on exactly one rank.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_partition_rows_equal_full_graph(world):
    import orientdb_amd as o
    scale = 9
    V = 1 << scale
    rp, col = o.rmat_csr(scale, 16, scale)
    trp, tcol = o.csr_transpose(V, rp, col)
    for r in range(world):
        lo, hi = o.partition_range(V, r, world)
        orp, ocol, irp, icol = o.rmat_partition(scale, lo, hi, 16, scale)
        assert len(orp) == hi - lo + 1 and len(irp) == hi - lo + 1
        assert np.array_equal(orp, rp[lo:hi + 1] - rp[lo])
        assert np.array_equal(ocol, col[rp[lo]:rp[hi]])
        assert np.array_equal(irp, trp[lo:hi + 1] - trp[lo])
        assert np.array_equal(icol, tcol[trp[lo]:trp[hi]])


def test_partition_raw_multigraph_rows():
    import orientdb_amd as o
    rp, col = o.rmat_csr(8, 16, 3, simple=False)
    orp, ocol, _, _ = o.rmat_partition(8, 64, 192, 16, 3, simple=False)
    assert np.array_equal(ocol, col[rp[64]:rp[192]])


def test_partitioned_snapshot_host_only():
    import orientdb_amd as o
    q = "MATCH {class:Person,as:a,where:(age < 1)}-Knows->{as:b}-Knows->{as:c,where:(age >= 90)} RETURN a,b,c"
    full = o.GraphSnapshot.rmat(9, device=-1)
    part = o.GraphSnapshot.rmat(9, device=-1, partition=(1, 4))
    assert part.part == (128, 256)
    assert o.OMatchStatement(q).explain(part) == o.OMatchStatement(q).explain(full)


def test_partition_range_validation():
    import orientdb_amd as o
    rp, col, irp, icol = o.rmat_partition(6, 0, 16)
    V = 64
    classes = [("V", -1, False, 9), ("E", -1, True, 10), ("Person", 0, False, 11), ("Knows", 1, True, 12)]
    es = [{"cls": 3, "out_rp": rp, "out_col": col, "in_rp": irp, "in_col": icol}]
    vc = np.full(V, 2, np.uint16)
    rids = np.arange(V, dtype=np.uint64)
    with pytest.raises(o.OmxError):  # row pointers of 16 rows declared as rows [0, 32)
        o.GraphSnapshot(V, classes, vc, rids, es, device=-1, part=(0, 32))
    with pytest.raises(o.OmxError):  # a partition without its in CSR
        o.GraphSnapshot(V, classes, vc, rids, [{"cls": 3, "out_rp": rp, "out_col": col}], device=-1, part=(0, 16))
    o.GraphSnapshot(V, classes, vc, rids, es, device=-1, part=(0, 16))


# ---- two gloo ranks: restatement of the exchange ---------------------------------------------------
SCALE = 10
QUERIES = [  # (name, query); filters and projections restated in _filters
    ("c2", "MATCH {class:Person,as:a,where:(age < 10)}-Knows->{as:b}-Knows->{as:c,where:(age >= 90)} RETURN a,b,c"),
    ("3hop", "MATCH {class:Person,as:a,where:(uid < 8)}-Knows->{as:b}-Knows->{as:c}-Knows->{as:d,where:(age<10)} RETURN a,b,c,d"),
    ("fof", "MATCH {class:Person,as:a,where:(age < 5)}-Knows->{as:b}-Knows->{as:c} RETURN a,c"),
]


def _filters(name, age, uid):
    if name == "c2":
        return age < 10, [None, age >= 90], (0, 1, 2)
    if name == "3hop":
        return uid < 8, [None, None, age < 10], (0, 1, 2, 3)
    return age < 5, [None, None], (0, 2)


def _partitioned_rows(rank, world, name, dist):
    """Rows of `name` on this rank: roots it owns, then per hop: expand through the local CSR, apply
    the target filter, route the new rows to owner(new vertex); finally route the projected tuples by
    hash and de-duplicate (exec.hip route_owner / route_hash, restated)."""
    import orientdb_amd as o
    V = 1 << SCALE
    lo, hi = o.partition_range(V, rank, world)
    orp, ocol, _, _ = o.rmat_partition(SCALE, lo, hi, 16, SCALE)
    age = o.synthetic_int_column(V, SCALE ^ 0xA9E, 100)
    uid = np.arange(V)
    root_f, hop_f, proj = _filters(name, age, uid)
    block = -(-V // world)
    rows = [(v,) for v in range(lo, hi) if root_f[v]]
    for h, f in enumerate(hop_f):
        out = []
        for r in rows:
            v = r[-1]
            assert lo <= v < hi, "a row reached a rank that does not own its source"
            for w in ocol[orp[v - lo]:orp[v - lo + 1]]:
                if f is None or f[w]:
                    out.append(r + (int(w),))
        if h + 1 < len(hop_f):  # the next hop reads row[-1]'s adjacency: owner routing
            buckets = [[] for _ in range(world)]
            for r in out:
                buckets[min(r[-1] // block, world - 1)].append(r)
            out = _exchange(buckets, rank, world, dist)
        rows = out
    tuples = [tuple(r[i] for i in proj) for r in rows]
    if name == "fof":  # distinct projection: hash routing, then a local distinct pass
        buckets = [[] for _ in range(world)]
        for t in tuples:
            buckets[hash(t) % world].append(t)
        tuples = sorted(set(_exchange(buckets, rank, world, dist)))
    return tuples


def _exchange(buckets, rank, world, dist):
    gathered = [None] * world
    dist.all_gather_object(gathered, buckets)
    return [tuple(r) for p in range(world) for r in gathered[p][rank]]


def _worker(rank, world, port, out):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        res = {name: _partitioned_rows(rank, world, name, dist) for name, _ in QUERIES}
        gathered = [None] * world
        dist.all_gather_object(gathered, res)
        if rank == 0:
            out.put(gathered)
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_rank_partitioned_exchange():
    import orientdb_amd as o
    from oracle import dfs
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    gathered = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    rp, col = o.rmat_csr(SCALE, 16, SCALE)
    V = 1 << SCALE
    age = o.synthetic_int_column(V, SCALE ^ 0xA9E, 100).astype(np.int64)
    cg = dfs.CsrGraph(rp, col, {"uid": np.arange(V, dtype=np.int64), "age": age})
    for name, query in QUERIES:
        r = dfs.run(cg, query, emit=True)
        cols = query.split("RETURN")[1].replace(" ", "").split(",")
        idx = [r["aliases"].index(c) for c in cols]
        want = {tuple(int(v) for v in row[idx]) for row in r["rows"]}
        shards = [set(g[name]) for g in gathered]
        assert set().union(*shards) == want, name
        if name == "fof":
            assert sum(len(s) for s in shards) == len(want)  # each distinct tuple on one rank
        assert all(len(g[name]) > 0 for g in gathered) or name == "3hop"


# ---- two gloo ranks: restatement of the partitioned multi-source BFS -------------------------------
def _msbfs_rows(rank, world, roots, depth, dist):
    """exec.hip varlen_msbfs on a partition, restated: every rank runs the batch of all roots (lanes);
    per level, prep over its own vertices (new = frontier & ~visited), an allgather of the owned frontier
    blocks, a pull over its own vertices' in-edges (OR of the in-neighbours' masks & ~visited); it emits
    (root, v) for its own visited vertices."""
    import orientdb_amd as o
    V = 1 << SCALE
    lo, hi = o.partition_range(V, rank, world)
    _, _, irp, icol = o.rmat_partition(SCALE, lo, hi, 16, SCALE)
    fr = np.zeros(V, np.uint64)
    vis = np.zeros(V, np.uint64)
    for i, r in enumerate(roots):
        fr[r] |= np.uint64(1) << np.uint64(i)
    for d in range(depth + 1):
        own = slice(lo, hi)
        new = fr[own] & ~vis[own]
        vis[own] |= new
        fr[:] = 0
        fr[own] = new
        if d == depth:
            break
        blocks = [None] * world
        dist.all_gather_object(blocks, (lo, hi, fr[own].copy()))
        for blo, bhi, b in blocks:
            fr[blo:bhi] = b
        if sum(int(np.count_nonzero(b)) for _, _, b in blocks) == 0:
            break
        nx = np.zeros(V, np.uint64)
        for v in range(lo, hi):
            acc = np.uint64(0)
            for u in icol[irp[v - lo]:irp[v - lo + 1]]:
                acc |= fr[u]
            nx[v] = acc & ~vis[v]
        fr = nx
    return [(int(roots[i]), v) for v in range(lo, hi) for i in range(len(roots))
            if (int(vis[v]) >> i) & 1]


def _msbfs_worker(rank, world, port, out):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        res = _msbfs_rows(rank, world, np.arange(40, dtype=np.uint32), 3, dist)
        gathered = [None] * world
        dist.all_gather_object(gathered, res)
        if rank == 0:
            out.put(gathered)
    finally:
        dist.destroy_process_group()


def test_two_rank_partitioned_msbfs():
    """The partitioned BFS's exchange (allgather of the owned frontier blocks) over two gloo ranks finds
    the oracle's BFS balls (oracle/bfs_ref.c) and emits each (root, v) on v's owner only."""
    import orientdb_amd as o
    from oracle import dfs
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_msbfs_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    gathered = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    rp, col = o.rmat_csr(SCALE, 16, SCALE)
    roots = np.arange(40, dtype=np.uint32)
    ref = dfs.bfs_varlen(rp, col, roots, max_depth=3, nthreads=2)
    want = {(int(roots[a]), int(b)) for a, b in ref["pairs"]}
    got = [set(g) for g in gathered]
    assert set().union(*got) == want
    assert sum(len(g) for g in gathered) == len(want)  # every (root, v) on one rank
    V = 1 << SCALE
    for r, g in enumerate(gathered):
        lo, hi = o.partition_range(V, r, world)
        assert all(lo <= v < hi for _, v in g)


# ---- two gloo ranks: restatement of the rank-0 projection (optional node, RETURN expressions, LIMIT) ---
DOC_Q = ("MATCH {class:Person,as:a,where:(uid < 200)}-Knows->{as:b, where:(age < 3), optional:true} "
         "RETURN a.uid as au, b.age as ba")


def _doc_rows(rank, world, dist):
    """exec.hip on a partition: the rank's roots; the optional hop on the owner of a (a row with no
    surviving neighbour continues with b = null, P/OMatchStatement.java:448-458); then every rank's rows
    go to rank 0 (route_rank0), which builds the documents from the replicated property columns and
    keeps the content-distinct ones (addResult :698-719)."""
    import orientdb_amd as o
    V = 1 << SCALE
    lo, hi = o.partition_range(V, rank, world)
    orp, ocol, _, _ = o.rmat_partition(SCALE, lo, hi, 16, SCALE)
    age = o.synthetic_int_column(V, SCALE ^ 0xA9E, 100)
    rows = []
    for a in range(lo, min(hi, 200)):
        bs = [int(w) for w in ocol[orp[a - lo]:orp[a - lo + 1]] if age[w] < 3]
        rows += [(a, b) for b in bs] if bs else [(a, None)]
    gathered = [None] * world
    dist.all_gather_object(gathered, rows)  # the all-to-all whose only destination is rank 0
    if rank != 0:
        return None
    docs = {(a, None if b is None else int(age[b])) for g in gathered for a, b in g}
    return sorted(docs, key=lambda d: (d[0], -1 if d[1] is None else d[1]))


def _doc_worker(rank, world, port, out):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        r = _doc_rows(rank, world, dist)
        if rank == 0:
            out.put(r)
    finally:
        dist.destroy_process_group()


def test_two_rank_documents_on_rank0():
    """The partitioned projection of RETURN expressions (documents by content, over the whole result:
    the rows of both gloo ranks meet on rank 0) equals the oracle's OResultSet on the full graph; LIMIT
    then cuts that one set (count only: which documents is HashSet-order-dependent, :404)."""
    import orientdb_amd as o
    from oracle.match_ref import MatchOracle
    from tests.rmat_oracle import refdb_from_csr
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_doc_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    docs = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    rp, col = o.rmat_csr(SCALE, 16, SCALE)
    age = o.synthetic_int_column(1 << SCALE, SCALE ^ 0xA9E, 100)
    want = MatchOracle(refdb_from_csr(rp, col, age), DOC_Q).execute()
    assert {(d["au"], d["ba"]) for d in want} == set(docs)
    assert len(want) == len(docs)
    assert any(d[1] is None for d in docs)  # the optional branch is exercised
    for limit in (1, 5):
        lim = MatchOracle(refdb_from_csr(rp, col, age), DOC_Q + " LIMIT %d" % limit).execute()
        assert len(lim) == min(limit, len(docs))
