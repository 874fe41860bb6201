"""The C++ planner (omx_statement_explain, host-only snapshot) reproduces the oracle's restatement of
estimateRootEntries / sortEdges / calculateMatch on every known-answer query, and declares as
device-executable exactly the queries tests/known_answers.py marks `gpu`."""
import pytest

from tests.known_answers import KNOWN
from oracle.match_ref import MatchOracle


@pytest.fixture(scope="module")
def host_graph(match_test_db_json):
    import orientdb_amd as o
    return o.GraphSnapshot.from_records(match_test_db_json, device=-1)


@pytest.mark.parametrize("case", KNOWN, ids=[k[0] for k in KNOWN])
def test_plan_matches_oracle(refdb, host_graph, case):
    import orientdb_amd as o
    name, line, query, params, outer, expect, gpu = case
    ref = MatchOracle(refdb, query).plan(params)
    st = o.OMatchStatement(query)
    got = st.explain(host_graph, *(params or []))
    assert got["estimates"] == ref["estimates"]
    assert got["prefetched"] == ref["prefetched"]
    assert got["root"] == ref["root"]
    assert [tuple(e) for e in got["edges"]] == [tuple(e) for e in ref["edges"]]
    assert got["supported"] == gpu, got["unsupported_reason"]


def test_rmat_plan_c2():
    """configs[1] query on a synthetic Person/Knows graph: root a (count/2), a→b, b→c forward."""
    import orientdb_amd as o
    g = o.GraphSnapshot.rmat(8, device=-1)
    st = o.OMatchStatement("MATCH {class:Person,as:a,where:(age < 1)}-Knows->{as:b}-Knows->{as:c,where:(age >= 90)} "
                           "RETURN a,b,c")
    p = st.explain(g)
    assert p["estimates"] == {"a": 128}
    assert p["root"] == "a" and p["edges"] == [["a", "b", True], ["b", "c", True]]
    assert p["supported"]
