"""Pins the full-size checker oracle/dfs_ref.c (driven by oracle/dfs.py run()) against the Python
oracle oracle/match_ref.py, which the reference's own OMatchStatementExecutionTest pins
(tests/test_oracle_known_answers.py). Every full-size parity claim (C1, C2, M1, C4, C5) rests on this
link: dfs_ref.c's DFS, reverse-edge filter rule, HashSet dedup of filtered forward hops
(P/OMatchPathItem.java:61,71-78) and digest are independent C code, so they are checked here against
the restatement of processContext (P/OMatchStatement.java:412-568) on small RMAT graphs, simple and
multigraph (parallel edges and self loops kept): the same result rows, the same complete bindings, the
same adjacency entries read (E_t) and, for rows distinct by construction, the same digest."""
import numpy as np
import pytest

from oracle.match_ref import MatchOracle, Record

QUERIES = [
    # RMAT_QUERIES / SEMI_QUERIES of tests/test_gpu_parity.py that dfs.run accepts
    ("c2_both_ends", "MATCH {class:Person,as:a,where:(age < 5)}-Knows->{as:b}-Knows->{as:c,where:(age >= 90)} RETURN a,b,c",
     ["a", "b", "c"]),
    ("c1_fof", "MATCH {class:Person}-Knows->{}-Knows->{as:fof} RETURN fof", ["fof"]),
    ("c1_abc", "MATCH {class:Person,as:a,where:(age < 20)}-Knows->{as:b}-Knows->{as:c} RETURN a,b,c", ["a", "b", "c"]),
    ("two_cols_dedup", "MATCH {class:Person,as:a,where:(age < 10)}-Knows->{as:b}-Knows->{as:c} RETURN a,c", ["a", "c"]),
    ("in_dir", "MATCH {class:Person,as:a,where:(age = 7)}<-Knows-{as:b}-Knows->{as:c,where:(age > 50)} RETURN a,b,c",
     ["a", "b", "c"]),
    ("both_dir", "MATCH {class:Person,as:a,where:(age = 3)}-Knows-{as:b,where:(age < 50)} RETURN a,b", ["a", "b"]),
    ("three_hop", "MATCH {class:Person,as:a,where:(uid < 8)}-Knows->{as:b}-Knows->{as:c}-Knows->{as:d,where:(age<10)} RETURN a,b,c,d",
     ["a", "b", "c", "d"]),
    ("triangle", "MATCH {class:Person,as:a}-Knows->{as:b}-Knows->{as:c}-Knows->{as:a} RETURN a,b,c", ["a", "b", "c"]),
    ("triangle_filtered", "MATCH {class:Person,as:a,where:(age < 30)}-Knows->{as:b}-Knows->{as:c,where:(age > 20)}-Knows->{as:a} RETURN a,b,c",
     ["a", "b", "c"]),
    ("matches", "MATCH {class:Person,as:a,where:(age = 11)}.out('Knows'){as:b}.out('Knows'){} RETURN $matches", ["a", "b"]),
    ("paths", "MATCH {class:Person,as:a,where:(age = 12)}.out('Knows'){as:b} RETURN $paths", ["a", "b"]),
    ("ab_of_abc", "MATCH {class:Person,as:a,where:(age < 5)}-Knows->{as:b}-Knows->{as:c,where:(age >= 90)} RETURN a, b",
     ["a", "b"]),
    ("a_of_abc", "MATCH {class:Person,as:a,where:(age < 20)}-Knows->{as:b}-Knows->{as:c,where:(age > 50)} RETURN a", ["a"]),
    ("three_hop_abc", "MATCH {class:Person,as:a,where:(uid < 8)}-Knows->{as:b}-Knows->{as:c}-Knows->{as:d,where:(age<10)} RETURN a, b, c",
     ["a", "b", "c"]),
    # a cycle-closing bound check from a small root set (the multigraph's parallel edges multiply the walks)
    ("triangle_small_roots", "MATCH {class:Person,as:a,where:(age < 6)}-Knows->{as:b}-Knows->{as:c,where:(age > 20)}-Knows->{as:a} RETURN a,b,c",
     ["a", "b", "c"]),
    # in / both hops with WHERE on the target (a forward, filtered, set-valued traversal)
    ("in_filtered", "MATCH {class:Person,as:a,where:(age < 8)}.in('Knows'){as:b,where:(age < 60)}.in('Knows'){as:c} RETURN a,b,c",
     ["a", "b", "c"]),
    ("both_two_hops", "MATCH {class:Person,as:a,where:(age = 4)}.both('Knows'){as:b}.both('Knows'){as:c,where:(age > 70)} RETURN a,b,c",
     ["a", "b", "c"]),
    # reverse edges (sortEdges starts from the cheaper end): the target's WHERE applies only in the free
    # branch (P/OMatchStatement.java:553-554), the traversal is executeReverse (no HashSet)
    ("reverse_free_where", "MATCH {class:Person,as:a,where:(age < 40)}-Knows->{as:b,where:(uid = 3)} RETURN a,b", ["a", "b"]),
    ("reverse_two_hops", "MATCH {class:Person,as:a,where:(age < 30)}-Knows->{as:b}-Knows->{as:c,where:(uid < 2)} RETURN a,b,c",
     ["a", "b", "c"]),
    ("reverse_both", "MATCH {class:Person,as:a,where:(age > 60)}-Knows-{as:b,where:(uid = 5)} RETURN a,b", ["a", "b"]),
    # a WHERE on a reversed target that has its own WHERE (estimate order puts the filtered end first)
    ("where_on_reversed_target", "MATCH {class:Person,as:a,where:(age >= 95)}<-Knows-{as:b,where:(uid < 3)} RETURN a,b",
     ["a", "b"]),
    # the WHERE of b declared on another occurrence of the alias: rebindFilters (P/OMatchStatement.java:185-195)
    # gives every item of the alias the merged filter, so the forward hop into b is filtered and set-valued
    ("where_on_other_occurrence", "MATCH {class:Person,as:a,where:(uid < 30)}-Knows->{as:b}, {as:b,where:(age < 50)} RETURN a,b",
     ["a", "b"]),
    ("where_split_over_occurrences", "MATCH {class:Person,as:a,where:(uid < 40)}-Knows->{as:b,where:(age > 10)}-Knows->{as:c},"
     " {as:b,where:(age < 70)} RETURN a,b,c", ["a", "b", "c"]),
]


def _graph(scale, simple):
    import orientdb_amd as o
    from oracle import dfs
    from tests.rmat_oracle import refdb_from_csr
    rp, col = o.rmat_csr(scale, 16, scale, simple)
    age = o.synthetic_int_column(1 << scale, scale ^ 0xA9E, 100).astype(np.int64)
    cg = dfs.CsrGraph(rp, col, {"uid": np.arange(1 << scale, dtype=np.int64), "age": age}, simple=simple)
    return cg, refdb_from_csr(rp, col, age)


_GRAPHS = {}


def graph(scale, simple):
    key = (scale, simple)
    if key not in _GRAPHS:
        _GRAPHS[key] = _graph(scale, simple)
    return _GRAPHS[key]


def _oracle(db, query):
    stats = {}
    rows = MatchOracle(db, query).execute(stats=stats)
    return rows, stats


def _rid(r):
    return (r.rid[0] << 48) | r.rid[1]


def _oracle_set(rows, cols):
    out = set()
    for r in rows:
        out.add((_rid(r),) if isinstance(r, Record) else tuple(_rid(r[c]) for c in cols))
    return out


@pytest.mark.parametrize("simple", [True, False], ids=["simple", "multigraph"])
@pytest.mark.parametrize("scale", [8, 9])
@pytest.mark.parametrize("q", QUERIES, ids=[q[0] for q in QUERIES])
def test_dfs_ref_equals_match_ref(q, scale, simple):
    from oracle import dfs
    name, query, cols = q
    if scale == 9 and name in ("c1_fof", "c1_abc", "triangle", "triangle_filtered", "two_cols_dedup"):
        pytest.skip("all-roots patterns: RMAT-8 only (the walk oracle is pure Python)")
    if not simple and (name in ("triangle", "triangle_filtered") or (scale == 9 and name.startswith("three_hop"))):
        pytest.skip("walks multiplied by parallel edges: triangle_small_roots and RMAT-8 cover the multigraph")
    cg, db = graph(scale, simple)
    want_rows, st = _oracle(db, query)
    r = dfs.run(cg, query, nthreads=4, digest=cols)
    idx = [r["aliases"].index(c) for c in cols]
    got = {tuple((11 << 48) | int(v) for v in row[idx]) for row in r["rows"]}
    want = _oracle_set(want_rows, cols)
    assert len(want) == len(want_rows)
    assert got == want
    assert r["bindings"] == st["bindings"], "complete matches before the de-duplication"
    assert r["edges"] == st.get("edges", 0), "adjacency entries read (E_t)"
    if len(cols) == len(r["aliases"]) and r["bindings"] == len(r["rows"]):
        # rows distinct by construction: the C sink's digest of every binding is the digest of the result
        assert r["digest"] == dfs.row_digest(np.array(sorted(want), np.uint64).reshape(-1, len(cols)))
    if len(cols) == 1:
        # one projected column: the C sink marks it in a V-bit set (the C1 full-size check), no rows kept
        d = dfs.run(cg, query, nthreads=4, emit=False, distinct=cols[0])
        assert {(11 << 48) | int(v) for v in d["distinct"]} == {w[0] for w in want}
        assert d["bindings"] == st["bindings"]


def test_pin_covers_both_graph_kinds():
    """The multigraph really has parallel edges and self loops, so the HashSet rule is exercised."""
    cg, _ = graph(8, False)
    src = np.repeat(np.arange(cg.V), np.diff(cg.rp).astype(np.int64))
    pairs = src.astype(np.int64) * cg.V + cg.col
    assert len(np.unique(pairs)) < len(pairs)
    assert np.any(src == cg.col)
