"""The 1-D partitioned MATCH on one MI355X: `world` partitions of one RMAT graph, each
rank a thread of this process with its own snapshot and stream on cuda:0, rows exchanged by the
thread transport (device-to-device copies) — the same routing code the RCCL transport drives across
GPUs. The union of the ranks' rows is compared bit-exactly with the oracle; RCCL itself is exercised
with a one-rank communicator routing through itself (OMX_ROUTE_SELF=1).
"""
import threading

import numpy as np
import pytest

from tests.test_gpu_parity import RMAT_QUERIES, _Ref, gpu_set

pytestmark = pytest.mark.gpu

DIST_IDS = ("c2_both_ends", "c1_fof", "c1_abc", "two_cols_dedup", "in_dir", "both_dir", "three_hop", "triangle",
            "triangle_filtered", "matches", "paths", "bound_candidate")
DIST_QUERIES = [q for q in RMAT_QUERIES if q[0] in DIST_IDS]


@pytest.fixture(scope="module")
def rmat10_full():
    import orientdb_amd as o
    g = o.GraphSnapshot.rmat(10, device=0, keep_csr=True)
    return g, _Ref(g, True)


_parts_cache = {}


def _parts(world):
    import orientdb_amd as o
    if world not in _parts_cache:
        _parts_cache[world] = [o.GraphSnapshot.rmat(10, device=0, partition=(r, world)) for r in range(world)]
    return _parts_cache[world]


def run_ranks(parts, query, **kw):
    """One thread per rank (ctypes releases the GIL inside omx_execute); returns the ranks' results."""
    import orientdb_amd as o
    comms = o.Comm.threads(len(parts))
    out, err = [None] * len(parts), []

    def work(r):
        try:
            out[r] = o.OMatchStatement(query).execute(parts[r], comm=comms[r], **kw)
        except BaseException as e:  # noqa: BLE001 — reported to the test thread
            err.append(e)

    th = [threading.Thread(target=work, args=(r,)) for r in range(len(parts))]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in th), "a rank did not finish (exchange deadlock)"
    for c in comms:
        c.close()
    if err:
        raise err[0]
    return out


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("q", DIST_QUERIES, ids=[q[0] for q in DIST_QUERIES])
def test_partitioned_parity(rmat10_full, world, q):
    _, ref = rmat10_full
    name, query, cols = q
    want = ref.expected(query, cols)
    res = run_ranks(_parts(world), query)
    got = [gpu_set(r, cols) for r in res]
    union = set().union(*got)
    assert union == want
    if name in ("c1_fof", "two_cols_dedup", "matches", "paths"):
        # distinct projections: the hash exchange puts each tuple on exactly one rank
        assert sum(len(g) for g in got) == len(want)


@pytest.mark.parametrize("world", [2, 3])
def test_partitioned_counts_match_replicated(rmat10_full, world):
    """COUNT mode: the ranks' edges/bindings add up to the single-snapshot run."""
    import orientdb_amd as o
    g, _ = rmat10_full
    for qn in ("c2_both_ends", "three_hop"):
        query = dict((x[0], x[1]) for x in RMAT_QUERIES)[qn]
        full = o.OMatchStatement(query).execute(g, mode=o.OMX_MODE_COUNT)
        res = run_ranks(_parts(world), query, mode=o.OMX_MODE_COUNT)
        assert sum(r.info["edges_traversed"] for r in res) == full.info["edges_traversed"]
        assert sum(r.info["bindings"] for r in res) == full.info["bindings"]
        assert sum(r.info["n_rows"] for r in res) == full.info["n_rows"]


def test_partitioned_sliced_kernel(rmat10_full, monkeypatch):
    """Filtered hops through the LDS-sliced heavy kernel on partitions (slice-cut index of owned rows)."""
    monkeypatch.setenv("OMX_HEAVY_DEG", "2")
    monkeypatch.setenv("OMX_SLICE_SHIFT", "7")
    _, ref = rmat10_full
    name, query, cols = [q for q in RMAT_QUERIES if q[0] == "c2_both_ends"][0]
    res = run_ranks(_parts(2), query)
    assert set().union(*[gpu_set(r, cols) for r in res]) == ref.expected(query, cols)


@pytest.mark.parametrize("world", [2, 3])
def test_partitioned_factorized(rmat10_full, world, monkeypatch):
    """The factorized expansion (distinct sources, grouped lists, rows over the lists) on every filtered
    hop of every rank: each rank decides on its own rows, which sit with the owner of their source."""
    import orientdb_amd as o
    monkeypatch.setenv("OMX_FACTOR", "force")
    _, ref = rmat10_full
    for lists in ("1", "0"):  # the lists through k_flists over each rank's own lists col, or binned
        monkeypatch.setenv("OMX_FLISTS", lists)
        for emit in ("force", "0"):
            monkeypatch.setenv("OMX_FEMIT", emit)
            for qn in ("c2_both_ends", "three_hop", "triangle_filtered", "in_dir"):
                name, query, cols = [q for q in RMAT_QUERIES if q[0] == qn][0]
                res = run_ranks(_parts(world), query, flags=o.OMX_FLAG_KERNEL_TIMING)
                assert set().union(*[gpu_set(r, cols) for r in res]) == ref.expected(query, cols), (qn, lists, emit)
                if qn == "c2_both_ends":
                    ran = {k["name"] for r in res for k in r.kernel_stats}
                    assert ("k_flists" in ran) == (lists == "1"), (lists, sorted(ran))


def test_rccl_one_rank_routes_through_itself(rmat10_full, monkeypatch):
    import orientdb_amd as o
    monkeypatch.setenv("OMX_ROUTE_SELF", "1")
    _, ref = rmat10_full
    part = o.GraphSnapshot.rmat(10, device=0, partition=(0, 1))
    comm = o.Comm.rccl(0, 1, 0, o.Comm.unique_id())
    try:
        for qn in ("c2_both_ends", "two_cols_dedup", "three_hop"):
            name, query, cols = [q for q in RMAT_QUERIES if q[0] == qn][0]
            rs = o.OMatchStatement(query).execute(part, comm=comm)
            assert gpu_set(rs, cols) == ref.expected(query, cols)
    finally:
        comm.close()


from tests.test_gpu_varlen import VARLEN  # noqa: E402

# variable-length and multi-step items on partitions: (row, vertex) pairs travel to the owner of their
# vertex every level (its adjacency is local there; all copies of a pair meet for the per-level dedup)
# and back to the rows' ranks at the end (exec.hip traverse / bind_pairs)
DIST_VARLEN = [q for q in VARLEN if q[0] in ("depth_only", "two_batches", "shared_sources", "where_target", "maxdepth",
                                             "maxdepth0", "while_prop", "in_dir", "both_dir", "where_depth",
                                             "bound_target")] + \
    [(q[0], q[1]) for q in RMAT_QUERIES if q[0] in ("multi_two_hops", "multi_varlen", "multi_edge_pair")]


def _vcols(q):
    return [c.strip() for c in q.split("RETURN")[1].split(",")]


@pytest.mark.parametrize("varlen", ["auto", "pairs"])
@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("q", DIST_VARLEN, ids=[q[0] for q in DIST_VARLEN])
def test_partitioned_varlen_parity(rmat10_full, world, q, varlen, monkeypatch):
    """auto: the BFS-exact items run the partitioned multi-source BFS (frontier blocks allgathered every
    level, rows emitted on the owner of their new vertex); pairs: (row, vertex) pairs routed per level."""
    import orientdb_amd as o
    if varlen == "pairs":
        monkeypatch.setenv("OMX_VARLEN", "pairs")
    g, ref = rmat10_full
    cols = _vcols(q[1])
    want = ref.expected(q[1], cols)
    res = run_ranks(_parts(world), q[1])
    got = [gpu_set(r, cols) for r in res]
    assert set().union(*got) == want
    assert sum(len(x) for x in got) == len(want)  # each row's result pairs end on the row's rank


@pytest.mark.parametrize("q", [q for q in DIST_VARLEN if q[0] in ("two_batches", "while_prop", "both_dir")],
                         ids=lambda q: q[0])
def test_partitioned_varlen_edges_match_replicated(rmat10_full, q, monkeypatch):
    """The partitioned traversal expands the same (row, vertex) frontiers as the replicated pair path."""
    import orientdb_amd as o
    g, _ = rmat10_full
    monkeypatch.setenv("OMX_VARLEN", "pairs")
    full = o.OMatchStatement(q[1]).execute(g)
    res = run_ranks(_parts(2), q[1])
    assert sum(r.info["edges_traversed"] for r in res) == full.info["edges_traversed"]
    assert sum(r.info["n_rows"] for r in res) == full.info["n_rows"]


@pytest.mark.parametrize("exchange", ["auto", "dense"])
@pytest.mark.parametrize("world", [2, 3, 4])
@pytest.mark.parametrize("q", [q for q in DIST_VARLEN if q[0] in ("depth_only", "two_batches", "while_prop", "both_dir",
                                                                  "where_target", "maxdepth")], ids=lambda q: q[0])
def test_partitioned_msbfs_matches_replicated(rmat10_full, q, world, exchange, monkeypatch):
    """The partitioned multi-source BFS (every level pulled over the rank's own vertices from the
    exchanged frontier: (vertex, mask) triples on sparse levels, whole blocks on dense ones — or always
    the blocks, OMX_DENSE_EXCHANGE=1) finds the replicated BFS's rows, level by level the same E_t."""
    import orientdb_amd as o
    g, _ = rmat10_full
    monkeypatch.setenv("OMX_VARLEN", "bfs")
    monkeypatch.setenv("OMX_DENSE_EXCHANGE", "1" if exchange == "dense" else "0")
    full = o.OMatchStatement(q[1]).execute(g, documents=False)
    res = run_ranks(_parts(world), q[1], documents=False)
    assert sum(r.info["edges_traversed"] for r in res) == full.info["edges_traversed"]
    assert sum(r.info["n_rows"] for r in res) == full.info["n_rows"]
    cols = _vcols(q[1])
    want = sorted(map(tuple, np.asarray(full.rows).tolist()))
    got = sorted(t for r in res for t in map(tuple, np.asarray(r.rows).tolist()))
    assert got == want and len(cols) == np.asarray(full.rows).shape[1]


def test_failing_rank_releases_its_peers(rmat10_full):
    """A rank whose execute fails (here: a missing query parameter on rank 0 only) aborts the thread
    communicator; its peer fails with an error instead of waiting forever in the exchange."""
    import orientdb_amd as o
    parts = _parts(2)
    comms = o.Comm.threads(2)
    q = RMAT_QUERIES[0][1]
    errs = [None, None]

    def work(r):
        try:
            o.OMatchStatement(q.replace("age < 5", "age < ?") if r == 0 else q).execute(parts[r], comm=comms[r])
        except o.OmxError as e:
            errs[r] = e

    th = [threading.Thread(target=work, args=(r,)) for r in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=60)
    assert not any(t.is_alive() for t in th), "the surviving rank hung in the exchange"
    assert errs[0] is not None and errs[1] is not None
    for c in comms:
        c.close()


def test_unsupported_keeps_communicator_usable(rmat10_full):
    """OMX_E_UNSUPPORTED before the first exchange is the host's 'run the reference engine' signal and
    is raised alike on every rank: it must not abort the communicator (ADVICE r2 capi.cpp), so the
    next supported query on the same Comm runs and matches the oracle."""
    import orientdb_amd as o
    _, ref = rmat10_full
    parts = _parts(2)
    comms = o.Comm.threads(2)
    name, query, cols = [q for q in RMAT_QUERIES if q[0] == "c2_both_ends"][0]
    unsup = "TRAVERSE out('Knows') FROM #11:0 STRATEGY DEPTH_FIRST"  # (the planner refuses it everywhere)
    out, errs = [None, None], [[], []]

    def work(r):
        try:
            for _ in range(2):
                try:
                    o.OMatchStatement(unsup).execute(parts[r], comm=comms[r])
                except o.OmxUnsupported as e:
                    errs[r].append(e)
            out[r] = o.OMatchStatement(query).execute(parts[r], comm=comms[r])
        except BaseException as e:  # noqa: BLE001
            errs[r].append(e)

    th = [threading.Thread(target=work, args=(r,)) for r in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in th)
    for c in comms:
        c.close()
    msg = [[type(x).__name__ + ": " + str(x) for x in e] for e in errs]
    assert all(len(e) == 2 and all(isinstance(x, o.OmxUnsupported) for x in e) for e in errs), msg[::-1]
    assert set().union(*[gpu_set(r, cols) for r in out]) == ref.expected(query, cols)


def test_partition_errors(rmat10_full):
    import orientdb_amd as o
    parts = _parts(2)
    with pytest.raises(o.OmxError):  # a partition needs its communicator
        o.OMatchStatement(RMAT_QUERIES[0][1]).execute(parts[0])
    comms = o.Comm.threads(2)
    with pytest.raises(o.OmxError):  # rank 1's communicator with rank 0's rows
        o.OMatchStatement(RMAT_QUERIES[0][1]).execute(parts[0], comm=comms[1])
    with pytest.raises(o.OmxError):  # the failed call aborted the communicator for every later one
        o.OMatchStatement(RMAT_QUERIES[0][1]).execute(parts[0], comm=comms[0])
    for c in comms:
        c.close()


# ---- partitioned coverage: optional nodes, RETURN expressions / JSON / $elements, LIMIT ---------------
from tests.test_gpu_parity import DOC_QUERIES, doc_set, oracle_rows  # noqa: E402

OPT_IDS = ("optional_free", "optional_bound", "elements", "paths", "matches")


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("q", [q for q in RMAT_QUERIES if q[0] in OPT_IDS], ids=lambda q: q[0])
def test_partitioned_optional_and_elements(rmat10_full, world, q):
    """Optional nodes (a row whose traversal finds nothing continues with the alias null, flagged on the
    owner of the source: P/OMatchStatement.java:448-458) and $elements / $paths / $matches on partitions;
    $elements is de-duplicated over the whole result, on rank 0 after every rank's rows met there."""
    _, ref = rmat10_full
    name, query, cols = q
    want = ref.expected(query, cols)
    res = run_ranks(_parts(world), query)
    cset = cols if cols and res[0].columns and res[0].columns[0] not in ("$elements", "$pathElements") else None
    got = [gpu_set(r, cset) for r in res]
    assert set().union(*got) == want
    assert sum(len(x) for x in got) == len(want)


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("q", DOC_QUERIES, ids=lambda q: q[0])
def test_partitioned_documents(rmat10_full, world, q):
    """RETURN expressions / JSON over a partitioned snapshot: every rank's rows meet on rank 0, which
    builds the documents from the replicated property columns and de-duplicates them by content
    (addResult :698-719, ODocumentEqualityWrapper); the other ranks return nothing. out()/in()/both() of
    an alias (out_list) reads lists rank 0 fetched from their owners (Executor::fetch_return_adjacency)."""
    g, ref = rmat10_full
    want = oracle_rows(ref.db, q[1])
    res = run_ranks(_parts(world), q[1])
    assert all(len(r) == 0 for r in res[1:])
    assert res[0].info["documents"] == 1
    assert doc_set(res[0]) == doc_set(want)
    # each rank de-duplicated its hash share of the alias tuples first: rank 0 received distinct tuples
    # only, at most the distinct bindings of every alias ($matches of the same pattern)
    import orientdb_amd as o
    head = q[1].split(" RETURN ")[0]
    m = o.OMatchStatement(head + " RETURN $matches").execute(g, documents=False)
    assert res[0].info["rows_gathered"] <= m.info["n_rows"]


def test_partitioned_return_adjacency_is_unsupported():
    """out()/in() of a list inside a RETURN expression (a.out('Knows').out('Knows')) reads lists whose
    vertices are only known while rank 0 evaluates it: refused alike on every rank before any exchange
    (the host runs the reference engine)."""
    import orientdb_amd as o
    q = "MATCH {class:Person,as:a,where:(uid < 15)} RETURN a.out('Knows').out('Knows').size() as d2"
    with pytest.raises(o.OmxUnsupported):
        run_ranks(_parts(2), q)


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("limit", [0, 1, 7, 100000])
def test_partitioned_limit(rmat10_full, world, limit):
    """LIMIT over the content-distinct result as a whole (OMatchStatement.java:741-746, LIMIT 0 = one row
    like addSingleResult :737-750): rank 0 returns min(max(limit, 1), total) distinct rows of the oracle's
    set, the others none."""
    _, ref = rmat10_full
    name, query, cols = [q for q in RMAT_QUERIES if q[0] == "c2_both_ends"][0]
    want = ref.expected(query, cols)
    res = run_ranks(_parts(world), query + " LIMIT %d" % limit)
    assert all(r.info["n_rows"] == 0 for r in res[1:])
    got = gpu_set(res[0], cols)
    assert len(got) == min(max(limit, 1), len(want))
    assert got <= want
    # every rank sent at most max(LIMIT, 1) of its distinct rows to rank 0
    assert res[0].info["rows_gathered"] <= min(world * max(limit, 1), len(want))


@pytest.mark.parametrize("limit", [0, 5, 10 ** 9])
def test_partitioned_count_limit(rmat10_full, limit):
    """COUNT mode with LIMIT on a partitioned snapshot: the ranks' counted rows are disjoint, so rank 0
    reports min(Σ ranks, max(LIMIT, 1)) (OMatchStatement.java:741-746), the others 0 — equal to the
    single-snapshot count under the same LIMIT."""
    import orientdb_amd as o
    g, _ = rmat10_full
    q = [x for x in RMAT_QUERIES if x[0] == "three_hop"][0][1] + " LIMIT %d" % limit
    full = o.OMatchStatement(q).execute(g, mode=o.OMX_MODE_COUNT, documents=False)
    res = run_ranks(_parts(3), q, mode=o.OMX_MODE_COUNT, documents=False)
    assert res[0].info["n_rows"] == full.info["n_rows"] == min(max(limit, 1), full.info["bindings"])
    assert all(r.info["n_rows"] == 0 for r in res[1:])


def test_partitioned_optional_null_reached_again_raises(rmat10_full):
    """The NPE of a null optional alias reached again (P/OMatchStatement.java:468) fails the partitioned
    execution on every rank (the rank that finds it aborts the exchanges of the others)."""
    import orientdb_amd as o
    q = ("MATCH {class:Person,as:a,where:(uid < 40)}-Knows->{as:b}-Knows->{as:c, where:(age < 30), optional:true},"
         "{as:a}-Knows->{as:c, optional:true} RETURN a, b, c")
    with pytest.raises(o.OmxError):
        run_ranks(_parts(2), q)


PART_EXTRA = [
    ("cartesian", [q for q in RMAT_QUERIES if q[0] == "cartesian"][0][1], ["a", "b"]),
    ("cartesian_after_hop", "MATCH {class:Person,as:a,where:(uid < 4)}-Knows->{as:c},{class:Person,as:b,where:(uid > 1018)} "
                            "RETURN a,b,c", ["a", "b", "c"]),
    ("degree_root", "MATCH {class:Person,as:a,where:(out('Knows').size() > 40)}-Knows->{as:b} RETURN a,b", ["a", "b"]),
    ("degree_target", "MATCH {class:Person,as:a,where:(uid < 30)}-Knows->{as:b,where:(in('Knows').size() < 3)} "
                      "RETURN a,b", ["a", "b"]),
    ("degree_both", "MATCH {class:Person,as:a,where:(both('Knows').size() = 20)}-Knows->{as:b} RETURN b", ["b"]),
]


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("q", PART_EXTRA, ids=lambda q: q[0])
def test_partitioned_cartesian_and_degrees(rmat10_full, world, q):
    """Disconnected patterns (a new root crossed with the rank's own rows: every vertex is a candidate,
    OMatchStatement.expandCartesianProduct :620-650) and out()/in()/both().size() predicates (the degrees
    of all ranks gathered once into global row pointers) on partitions."""
    _, ref = rmat10_full
    name, query, cols = q
    want = ref.expected(query, cols)
    res = run_ranks(_parts(world), query)
    got = [gpu_set(r, cols) for r in res]
    assert set().union(*got) == want and len(want) > 0


# ---- partitioned TRAVERSE / SELECT expand() / shortestPath(): rank 0 walks, the owners serve lists ----
def _chain_queries(g):
    rp = g.csr[0].astype(np.int64)
    deg = np.diff(rp)
    hub, leaf = int(np.argmax(deg)), int(np.argmax(deg == 1))
    return [
        ("traverse_while", "TRAVERSE out('Knows') FROM #11:%d WHILE $depth < 3 STRATEGY BREADTH_FIRST" % hub),
        ("traverse_maxdepth", "TRAVERSE out('Knows') FROM [#11:3, #11:7, #11:3] MAXDEPTH 2 STRATEGY BREADTH_FIRST"),
        ("traverse_limit_both", "TRAVERSE both('Knows') FROM #11:%d MAXDEPTH 3 LIMIT 50 STRATEGY BREADTH_FIRST" % leaf),
        ("traverse_prop", "TRAVERSE in('Knows') FROM #11:%d WHILE age < 70 STRATEGY BREADTH_FIRST" % hub),
        ("select_chain", "SELECT expand(out('Knows').out('Knows')) FROM #11:%d" % hub),
        ("select_where", "SELECT expand(in('Knows').out('Knows')) FROM Person WHERE uid < 20"),
        ("shortest_out", "SELECT expand(shortestPath(#11:%d, #11:%d, 'OUT', 'Knows'))" % (leaf, hub)),
        ("shortest_both", "SELECT expand(shortestPath(#11:%d, #11:%d, 'BOTH'))" % (hub, leaf)),
    ]


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("qi", range(8), ids=["traverse_while", "traverse_maxdepth", "traverse_limit_both", "traverse_prop",
                                              "select_chain", "select_where", "shortest_out", "shortest_both"])
def test_partitioned_chains(rmat10_full, world, qi):
    """TRAVERSE / SELECT expand() / shortestPath() on a partitioned snapshot (Executor::serve_chain): rank 0
    runs the ordered walk over lists its peers fetch from their rows, so the records come in the
    reference's order, equal to the single-snapshot run's; the other ranks return nothing."""
    import orientdb_amd as o
    g, _ = rmat10_full
    name, q = _chain_queries(g)[qi]
    full = o.OMatchStatement(q).execute(g, documents=False)
    res = run_ranks(_parts(world), q, documents=False)
    assert np.array_equal(np.asarray(res[0].rows), np.asarray(full.rows)), name
    assert res[0].info["edges_traversed"] == full.info["edges_traversed"]
    assert all(r.info["n_rows"] == 0 for r in res[1:])
