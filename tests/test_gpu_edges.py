"""Edge nodes on a snapshot with edge records (include/omx/match.h omx_edge_set_desc.edge_rids): MATCH binds
edge records — outE('L'){as: e, where: (...)}.inV(), inE().outV(), bothE().bothV(), edge-class roots,
reversed edge items (executeReverse: outE ↔ outV, inE ↔ inV, P/OMethodCall.java:92-126), $paths /
$pathElements with the edge records, RETURN expressions over edge fields — checked against the Python
oracle (oracle/match_ref.py, whose RefDB keeps regular edges as records, B/OrientVertex.java:109-180).

Two graphs: the reference's known-answer database (tests/golden/match_test_db.json) with its edges as
records — every known-answer case the device runs must give the same rows as on the lightweight snapshot —
and a seeded Person graph whose Knows / Likes edges carry fields (since, w, tag; some absent).
"""
import numpy as np
import pytest

from oracle.match_ref import MatchOracle, RefDB
from tests.known_answers import KNOWN
from tests.test_gpu_parity import doc_set, gpu_set, oracle_set

pytestmark = pytest.mark.gpu


def edge_db(n=160, n_knows=900, n_likes=300, seed=5):
    """Record-level description (tests/golden/make_match_test_db.py's JSON shape) with edge fields."""
    rng = np.random.default_rng(seed)
    classes = [{"name": "V", "superclass": None, "is_edge": False}, {"name": "E", "superclass": None, "is_edge": True},
               {"name": "Person", "superclass": "V", "is_edge": False},
               {"name": "Knows", "superclass": "E", "is_edge": True},
               {"name": "Likes", "superclass": "E", "is_edge": True}]
    verts = [{"class": "Person", "props": {"uid": i, "age": int(rng.integers(0, 100))}} for i in range(n)]
    edges = []
    for k in range(n_knows):
        a, b = (int(x) for x in rng.integers(0, n, 2))
        props = {"since": int(rng.integers(2005, 2021)), "w": float(rng.random())}
        if k % 3:
            props["tag"] = ["x", "y", "z"][k % 5 % 3]
        edges.append({"class": "Knows", "out": a, "in": b, "props": props})
    for k in range(n_likes):
        a, b = (int(x) for x in rng.integers(0, n, 2))
        edges.append({"class": "Likes", "out": a, "in": b, "props": {"since": int(rng.integers(2010, 2021))}})
    return {"classes": classes, "vertices": verts, "edges": edges, "indexes": []}


@pytest.fixture(scope="module")
def edb():
    import orientdb_amd as o
    d = edge_db()
    return o.GraphSnapshot.from_records(d, device=0, edge_records=True), RefDB.from_json(d)


@pytest.fixture(scope="module")
def kdb(match_test_db_json):
    import orientdb_amd as o
    return o.GraphSnapshot.from_records(match_test_db_json, device=0, edge_records=True)


EDGE_QUERIES = [
    "MATCH {class: Person, as: a, where: (age < 40)}.outE('Knows'){as: e, where: (since > 2012)}.inV(){as: b} RETURN a, e, b",
    "MATCH {class: Person, as: a}.outE('Knows'){as: e, where: (w < 0.3)}.inV(){as: b, where: (age > 50)} RETURN e",
    "MATCH {class: Person, as: a, where: (uid < 20)}.inE('Knows'){as: e}.outV(){as: b} RETURN a, e, b",
    "MATCH {class: Knows, as: e, where: (since = 2015)}.outV(){as: a} RETURN e, a",
    "MATCH {class: Knows, as: e, where: (since = 2015)}.inV(){as: b}.outE('Likes'){as: f}.inV(){as: c} RETURN e, f, c",
    "MATCH {class: Person, as: a, where: (uid = 7)}.bothE(){as: e}.bothV(){as: b} RETURN e, b",
    "MATCH {class: Person, as: a, where: (uid < 30)}.outE('Knows'){as: e}.inV(){as: b}, "
    "{as: b}.outE('Knows'){as: f}.inV(){as: a} RETURN a, b, e, f",
    "MATCH {class: Person, as: a, where: (uid < 50)}.outE('Knows'){as: e, where: (tag = 'x')}.inV(){as: b} RETURN $elements",
    "MATCH {class: Person, as: a, where: (uid < 50)}.outE('Knows'){as: e, where: (tag = 'x')}.inV(){as: b} RETURN $pathElements",
    "MATCH {class: Person, as: a, where: (uid < 30)}.outE('Knows').inV(){as: b}.outE('Likes').inV(){as: c} RETURN $paths",
    "MATCH {class: Person, as: a, where: (uid < 30)}.outE('Knows'){as: e}.inV(){as: b} RETURN $matches",
    "MATCH {class: Person, as: a, where: (uid < 25)}.outE('Knows'){as: e, optional: true, where: (since > 2018)} RETURN a, e",
    "MATCH {class: Person, as: a, where: (uid < 40)}.outE(){as: e, class: Likes}.inV(){as: b} RETURN e, b",
    "MATCH {class: Person, as: a, where: (uid < 40)}.outE('Knows'){as: e}.inV(){as: b} RETURN e.since AS s, a.uid AS u, e.tag AS t",
    "MATCH {class: Person, as: b, where: (uid < 40)}.inE('Knows'){as: e, where: (since > 2015)}.outV(){as: a, where: (age < 50)} RETURN a, e",
    "MATCH {class: Person, as: a, where: (uid < 60)}.outE('Knows'){as: e}.inV(){as: b, where: ($matched.a != $currentMatch)} RETURN e",
    "MATCH {as: a}.outE('Knows'){as: e, class: Knows, where: (since = 2013)}.inV(){as: b} RETURN a, e, b",
    "MATCH {as: a, class: Person}.outE('Knows'){as: e}.inV(){as: b, class: Person, where: (uid = 3)} RETURN a, e",
    "MATCH {class: Person, as: a, where: (uid < 30)}.outE('Knows'){as: e}, {as: e}.inV(){as: b} RETURN a, e, b",
    "MATCH {class: Person, as: a, where: (uid < 30)}.outE('Knows'){as: e}.inV(){as: b}.out('Likes'){as: c} RETURN e, c",
    "MATCH {class: Likes, as: f}.inV(){as: b, where: (age < 20)} RETURN f",
    "MATCH {class: E, as: e, where: (since = 2020)} RETURN e",
    # the edge documents' `out` / `in` links (ODocument fields of a regular edge)
    "MATCH {class: Person, as: a, where: (uid < 30)}.outE('Knows'){as: e, where: (since > 2015)}.inV(){as: b} "
    "RETURN e.out AS o, e.in AS i, e.since AS s",
    "MATCH {class: Knows, as: e, where: (since = 2015)} RETURN e.out.uid AS u, e.in.age AS g, e.w AS w",
]


def _check(g, ref, query):
    import orientdb_amd as o
    rs = o.OMatchStatement(query).execute(g)
    want = MatchOracle(ref, query).execute()
    assert rs.info["n_rows"] == len(want)
    if rs.info["documents"]:
        assert doc_set(rs) == doc_set(want)
        return rs
    cols = rs.columns if rs.columns[0] not in ("$elements", "$pathElements") else None
    assert gpu_set(rs) == oracle_set(want, cols)
    return rs


@pytest.mark.parametrize("query", EDGE_QUERIES, ids=[f"q{i}" for i in range(len(EDGE_QUERIES))])
def test_edge_nodes(edb, query):
    g, ref = edb
    rs = _check(g, ref, query)
    assert rs.info["n_rows"] > 0 or "optional" in query  # every case has matches on this graph


def test_edge_nodes_count_mode(edb):
    import orientdb_amd as o
    g, ref = edb
    q = EDGE_QUERIES[0]
    rs = o.OMatchStatement(q).execute(g, mode=o.OMX_MODE_COUNT)
    assert rs.info["n_rows"] == len(MatchOracle(ref, q).execute())


def test_edge_nodes_unsupported_on_lightweight(match_test_db_json):
    import orientdb_amd as o
    g = o.GraphSnapshot.from_records(match_test_db_json, device=0)
    with pytest.raises(o.OmxUnsupported):
        o.OMatchStatement("MATCH {class: TriangleV, as: a}.outE('TriangleE'){as: e}.inV(){as: b} RETURN a, e, b").execute(g)


GPU_CASES = [k for k in KNOWN if k[6]]


@pytest.mark.parametrize("case", GPU_CASES, ids=[k[0] for k in GPU_CASES])
def test_known_answers_with_edge_records(refdb, kdb, case):
    """The same rows as the lightweight snapshot's (test_gpu_parity) with the edges as records."""
    import orientdb_amd as o
    name, line, query, params, outer, expect, _ = case
    ref = MatchOracle(refdb, query).execute(params)
    rs = o.OMatchStatement(query).execute(kdb, *(params or []))
    assert rs.info["n_rows"] == len(ref)
    if "limit" in query.lower():
        return
    if rs.info["documents"]:
        assert doc_set(rs) == doc_set(ref)
        return
    cols = rs.columns if rs.columns[0] not in ("$elements", "$pathElements") else None
    assert gpu_set(rs) == oracle_set(ref, cols)


KNOWN_DB_EDGE_QUERIES = [
    "match {class:TriangleV, as: friend1}.outE('TriangleE').inV(){as: friend2, where: (uid = 1)}"
    ".outE('TriangleE').inV(){as: friend3} return $paths",
    "match {class:TriangleV, as: friend1}.outE('TriangleE'){as: e}.inV(){as: friend2, where: (uid = 1)} return $pathElements",
    "match {class:Employee, as: m}.outE('ManagerOf'){as: e}.inV(){as: d}.inE('ParentDepartment'){as: p}.outV(){as: c} return e, p, c",
    "match {class:IndexedEdge, as: e} return e",
]


@pytest.mark.parametrize("query", KNOWN_DB_EDGE_QUERIES, ids=[f"k{i}" for i in range(len(KNOWN_DB_EDGE_QUERIES))])
def test_known_db_edge_nodes(refdb, kdb, query):
    """Edge nodes and $paths / $pathElements with edge steps on the known-answer database (left to the
    reference engine on the lightweight snapshot)."""
    rs = _check(kdb, refdb, query)
    assert rs.info["n_rows"] > 0


# ---- RMAT snapshots with edge records (GraphSnapshot.rmat(edge_records=True): RID #12:i, field w) ------
@pytest.fixture(scope="module")
def rmat_edges():
    import orientdb_amd as o
    from tests.rmat_oracle import refdb_from_csr
    g = o.GraphSnapshot.rmat(10, device=0, keep_csr=True, edge_records=True)
    return g, refdb_from_csr(g.csr[0], g.csr[1], g.age, g.w)


RMAT_EDGE_QUERIES = [
    "MATCH {class:Person,as:a,where:(age < 5)}.outE('Knows'){as:e, where:(w < 30)}.inV(){as:b,where:(age >= 50)} RETURN a, e, b",
    "MATCH {class:Person,as:a,where:(uid < 40)}.inE('Knows'){as:e, where:(w >= 90)}.outV(){as:b} RETURN a, e, b",
    "MATCH {class:Knows,as:e,where:(w = 7)}.inV(){as:b,where:(age < 50)} RETURN e, b",
    "MATCH {class:Person,as:a,where:(uid < 30)}.outE('Knows'){as:e, where:(w < 20)}.inV(){as:b}.out('Knows'){as:c,where:(age < 10)} RETURN a, e, b, c",
    "MATCH {class:Person,as:a,where:(uid < 20)}.outE('Knows'){as:e, where:(w < 50)}.inV(){as:b} RETURN $pathElements",
    "MATCH {class:Person,as:a,where:(uid < 50)}.bothE('Knows'){as:e, where:(w < 5)}.bothV(){as:b} RETURN a, e, b",
]


@pytest.mark.parametrize("query", RMAT_EDGE_QUERIES, ids=[f"r{i}" for i in range(len(RMAT_EDGE_QUERIES))])
def test_rmat_edge_nodes(rmat_edges, query):
    g, db = rmat_edges
    rs = _check(g, db, query)
    assert rs.info["n_rows"] > 0


def test_e1_rmat20_vs_edge_ref():
    """The E1 bench line's shape at RMAT-20, whole result: rows, E_t and the digest of the (a, e, b) RID
    rows against oracle/edge_ref.py (pinned to match_ref.py by tests/test_oracle_edge_ref.py)."""
    import numpy as np
    import orientdb_amd as o
    from oracle.dfs import row_digest
    from oracle.edge_ref import edge_two_hop
    g = o.GraphSnapshot.rmat(20, device=0, keep_csr=True, edge_records=True)
    q = ("MATCH {class:Person,as:a,where:(age < 1)}.outE('Knows'){as:e, where:(w < 10)}.inV(){as:b,where:(age >= 90)} "
         "RETURN a, e, b")
    (a, e, b), edges = edge_two_hop(g.csr[0], g.csr[1], np.nonzero(g.age < 1)[0], g.w < 10, g.age >= 90)
    want = row_digest(np.stack([(np.uint64(11) << np.uint64(48)) | a.astype(np.uint64),
                                (np.uint64(12) << np.uint64(48)) | e.astype(np.uint64),
                                (np.uint64(11) << np.uint64(48)) | b.astype(np.uint64)], axis=1))
    rs = o.OMatchStatement(q).execute(g, flags=o.OMX_FLAG_KEEP_DEVICE | o.OMX_FLAG_DIGEST, documents=False)
    assert rs.info["n_rows"] == len(a) > 1000
    assert rs.info["edges_traversed"] == edges
    assert rs.info["digest"] == want
