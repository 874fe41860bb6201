"""TRAVERSE / SELECT expand() statements: parsing and which forms the device engine takes (CPU, host-only
snapshot). The supported forms are the BREADTH_FIRST work list over out()/in()/both() fields and
expand() chains of moves; everything else is reported unsupported so the host keeps the reference
executor (S/OCommandExecutorSQLTraverse.java, S/OCommandExecutorSQLSelect.java).
"""
import pytest

import orientdb_amd as o


@pytest.fixture(scope="module")
def g():
    return o.GraphSnapshot.rmat(8, device=-1)


CASES = [
    ("TRAVERSE out('Knows') FROM #11:3 WHILE $depth < 3 STRATEGY BREADTH_FIRST", True, "TRAVERSE"),
    ("traverse in('Knows') from [#11:3, #11:4] maxdepth 2 limit 10 strategy breadth_first", True, "TRAVERSE"),
    ("TRAVERSE both() FROM Person WHILE age < 50 and $depth <= 2 STRATEGY BREADTH_FIRST", True, "TRAVERSE"),
    ("TRAVERSE out('Knows') FROM #11:3 WHERE $depth < 2 STRATEGY BREADTH_FIRST", True, "TRAVERSE"),  # deprecated WHERE
    ("TRAVERSE out('Knows'), out('Knows') FROM #11:3 STRATEGY BREADTH_FIRST", True, "TRAVERSE"),  # a Set of fields
    ("TRAVERSE out('Knows') FROM #11:3 WHILE $depth < 3", False, "TRAVERSE"),  # DEPTH_FIRST (default)
    ("TRAVERSE * FROM #11:3 STRATEGY BREADTH_FIRST", False, "TRAVERSE"),
    ("TRAVERSE any() FROM #11:3 STRATEGY BREADTH_FIRST", False, "TRAVERSE"),
    ("TRAVERSE out_Knows FROM #11:3 STRATEGY BREADTH_FIRST", False, "TRAVERSE"),
    ("TRAVERSE out('Knows'), in('Knows') FROM #11:3 STRATEGY BREADTH_FIRST", False, "TRAVERSE"),  # HashSet order
    ("TRAVERSE out() FROM (select from Person) STRATEGY BREADTH_FIRST", False, "TRAVERSE"),
    ("TRAVERSE out() FROM cluster:person STRATEGY BREADTH_FIRST", False, "TRAVERSE"),
    ("TRAVERSE out() FROM #11:3 SKIP 2 STRATEGY BREADTH_FIRST", False, "TRAVERSE"),
    ("TRAVERSE out() FROM #11:3 WHILE $depth < 2.5 STRATEGY BREADTH_FIRST", False, "TRAVERSE"),  # Integer conversion
    ("SELECT expand(out('Knows').out('Knows')) FROM #11:0", True, "SELECT"),
    ("SELECT expand(outE('Knows').inV()) FROM Person WHERE uid < 3 LIMIT 5", True, "SELECT"),
    ("SELECT expand(in()) FROM [#11:1, #11:2]", True, "SELECT"),
    ("SELECT expand(out('Knows').name) FROM #11:0", False, "SELECT"),
    ("SELECT expand(bothE().bothV()) FROM #11:0", False, "SELECT"),
    ("SELECT expand(out())", False, "SELECT"),  # no FROM
    ("SELECT shortestPath(#11:1, #11:9)", True, "SHORTEST_PATH"),
    ("SELECT shortestPath(#11:1, #11:9, 'OUT', 'Knows') AS p", True, "SHORTEST_PATH"),
    ("SELECT expand(shortestPath(#11:1, #11:9, 'both', null, {'maxDepth': 3}))", True, "SHORTEST_PATH"),
    ("SELECT expand(shortestPath(?, ?, 'IN'))", True, "SHORTEST_PATH"),
    ("SELECT shortestPath(#11:1, #11:9) FROM Person", False, "SHORTEST_PATH"),
    ("SELECT shortestPath(#11:1, out())", False, "SHORTEST_PATH"),
]


@pytest.mark.parametrize("q,supported,kind", CASES, ids=[c[0][:60] for c in CASES])
def test_chain_support(g, q, supported, kind):
    p = o.OMatchStatement(q).explain(g, *(["#11:1", "#11:9"] if "?" in q else []))
    assert p["kind"] == kind
    assert p["supported"] == supported, p["unsupported_reason"]


def test_parse_errors():
    for q in ["TRAVERSE FROM #11:3", "TRAVERSE out() #11:3", "TRAVERSE out() FROM #11:0 LIMIT 0",
              "TRAVERSE out() FROM #11:0 STRATEGY SIDEWAYS", "TRAVERSE out() FROM #11"]:
        with pytest.raises(o.OmxParseError):
            o.OMatchStatement(q)
    with pytest.raises(o.OmxUnsupported):
        o.OMatchStatement("SELECT FROM Person")


def test_unknown_class_is_an_execution_error(g):
    with pytest.raises(o.OmxExecutionError):
        o.OMatchStatement("TRAVERSE out() FROM Nope STRATEGY BREADTH_FIRST").explain(g)


def test_legacy_null_semantics(g):
    # a condition on a field no vertex has: every comparison is false in the legacy filter, != included
    # (OQueryOperatorEqualityNotNulls), so != cannot take the device's null semantics
    ok = o.OMatchStatement("TRAVERSE out() FROM #11:0 WHILE nope > 3 STRATEGY BREADTH_FIRST").explain(g)
    assert ok["supported"], ok["unsupported_reason"]
    ne = o.OMatchStatement("TRAVERSE out() FROM #11:0 WHILE nope <> 3 STRATEGY BREADTH_FIRST").explain(g)
    assert not ne["supported"]


def test_match_edge_steps_fuse(g):
    q = "MATCH {class:Person, as:a, where:(uid = 1)}.outE('Knows').inV(){as:b} RETURN a, b"
    assert o.OMatchStatement(q).explain(g)["supported"]
    q2 = "MATCH {class:Person, as:a, where:(uid = 1)}.outE('Knows').inV(){as:b} RETURN $paths"
    assert not o.OMatchStatement(q2).explain(g)["supported"]
    q3 = "MATCH {class:Person, as:a, where:(uid = 1)}.outE('Knows'){as:e}.inV(){as:b} RETURN a, b"
    assert not o.OMatchStatement(q3).explain(g)["supported"]


def test_shortest_path_bad_direction(g):
    with pytest.raises(o.OmxExecutionError):
        o.OMatchStatement("SELECT shortestPath(#11:1, #11:9, 'SIDEWAYS')").explain(g)
