"""Pins the oracle (oracle/match_ref.py) against every known-answer assertion of the reference's
OMatchStatementExecutionTest (see tests/known_answers.py for the line of each)."""
import pytest

from tests.known_answers import KNOWN
from oracle.match_ref import MatchOracle, Record


def check_outer(db, rows, outer, expect):
    count, values = expect
    if count is not None:
        assert len(rows) == count, rows
    if outer is None:
        return
    kind, key = outer
    if kind == "names":
        names = [r[key].props.get("name") for r in rows]
        if values is not None:
            assert set(names) == values
    elif kind == "names_not":
        names = [r[key].props.get("name") for r in rows]
        assert not (set(names) & values)
    elif kind == "field":
        assert {r[key] for r in rows} == values
    elif kind == "uids":
        assert {tuple(r[a].props["uid"] for a in key) for r in rows} == values
    elif kind == "uid_of":
        assert {r[key].props["uid"] for r in rows} == values
    elif kind == "record_names":
        assert all(isinstance(r, Record) for r in rows)
        assert {r.props.get("name") for r in rows} == values
    elif kind == "field_kind":
        assert all(isinstance(r[key], Record) and not r[key].is_edge for r in rows)
    elif kind == "field_len":
        assert all(len(r[key]) == values for r in rows)
    elif kind == "list_uids":  # a list of vertices whose uids are `values`, in order
        assert all([x.props["uid"] for x in r[key]] == values for r in rows)
    elif kind == "field_prefix":
        assert all(str(r[key]).startswith(values) for r in rows)
    else:
        raise AssertionError(kind)


@pytest.mark.parametrize("case", KNOWN, ids=[k[0] for k in KNOWN])
def test_known_answer(refdb, case):
    name, line, query, params, outer, expect, _gpu = case
    rows = MatchOracle(refdb, query).execute(params)
    check_outer(refdb, rows, outer, expect)


def test_triangle_cycles_derived(refdb):
    """SURVEY Appendix B derived fixture: directed 3-cycles {0→2→4→0} and {8→4→7→8} → 6 rotations."""
    q = ("match {class:TriangleV,as:a}-TriangleE->{as:b}-TriangleE->{as:c}-TriangleE->{as:a} return a, b, c")
    rows = MatchOracle(refdb, q).execute()
    got = {tuple(r[x].props["uid"] for x in "abc") for r in rows}
    assert got == {(0, 2, 4), (2, 4, 0), (4, 0, 2), (8, 4, 7), (4, 7, 8), (7, 8, 4)}


def test_plan_triangle(refdb):
    """sortEdges on a cycle: a→b forward, c→a reversed, b→c forward-closing."""
    q = "match {class:TriangleV,as:a}-TriangleE->{as:b}-TriangleE->{as:c}-TriangleE->{as:a} return a, b, c"
    plan = MatchOracle(refdb, q).plan()
    assert plan["root"] == "a"
    assert plan["edges"] == [("a", "b", True), ("c", "a", False), ("b", "c", True)]
