"""Parity of the HIP path (through the C-ABI) with the oracle: bit-exact sets of RID tuples.

* every known-answer case of the reference's OMatchStatementExecutionTest the device engine executes;
* RMAT Person/Knows graphs (SURVEY §8(d) schema) at oracle-sized scales: 2-hop with WHERE on both
  ends (configs[1] shape), single-alias projections (dedup), $elements, both()/in(), triangles
  (cycle closing, configs[3] shape), variable-length while/maxDepth (configs[2] shape), cartesian,
  root sharding (the multi-GPU partition) and COUNT mode.
"""
import numpy as np
import pytest

from tests.known_answers import KNOWN
from oracle.match_ref import MatchOracle, Record

pytestmark = pytest.mark.gpu


def oracle_rows(db, query, params=None, limit=None):
    return MatchOracle(db, query).execute(params, limit)


NULL_RID = (1 << 64) - 1  # an unmatched optional node (include/omx/match.h OMX_NULL_RID)


def oracle_set(rows, cols):
    out = set()
    for r in rows:
        if isinstance(r, Record):
            out.add(((r.rid[0] << 48) | r.rid[1],))
        else:
            out.add(tuple(NULL_RID if r[c] is None else (r[c].rid[0] << 48) | r[c].rid[1] for c in cols))
    return out


def gpu_set(rs, cols=None):
    if rs.rows.shape[0] == 0:
        return set()
    idx = [rs.columns.index(c) for c in cols] if cols else list(range(rs.rows.shape[1]))
    s = {tuple(int(x) for x in row[idx]) for row in rs.rows}
    assert len(s) == rs.rows.shape[0], "device result has duplicate rows"
    return s


@pytest.fixture(scope="module")
def gdb(match_test_db_json):
    import orientdb_amd as o
    return o.GraphSnapshot.from_records(match_test_db_json, device=0)


GPU_CASES = [k for k in KNOWN if k[6]]


@pytest.mark.parametrize("case", GPU_CASES, ids=[k[0] for k in GPU_CASES])
def test_known_answers_on_device(refdb, gdb, case):
    import orientdb_amd as o
    name, line, query, params, outer, expect, _ = case
    ref = oracle_rows(refdb, query, params)
    rs = o.OMatchStatement(query).execute(gdb, *(params or []))
    count = expect[0]
    if count is not None:
        assert rs.info["n_rows"] == count
    assert rs.info["n_rows"] == len(ref)
    if "limit" in query.lower():
        return  # LIMIT picks HashSet-order-dependent rows (OMatchStatement.java:404): count only
    if rs.info["documents"]:  # RETURN expressions / JSON: documents equal by content
        assert doc_set(rs) == doc_set(ref)
        return
    cols = rs.columns if rs.columns[0] not in ("$elements", "$pathElements") else None
    assert gpu_set(rs) == oracle_set(ref, cols)


def _norm(x):
    """Content of a result value: records by RID, documents by their fields (ODocumentEqualityWrapper)."""
    if isinstance(x, Record):
        return ("r", tuple(x.rid))
    if x is not None and type(x).__name__ == "ORecordId":
        return ("r", tuple(x))
    if isinstance(x, dict):
        return ("d", tuple(sorted((k, _norm(v)) for k, v in x.items())))
    if isinstance(x, (list, tuple)):
        return ("l", tuple(_norm(v) for v in x))
    return ("v", x)


def doc_set(rows):
    out = {_norm(r) for r in rows}
    assert len(out) == len(rows), "duplicate documents"
    return out


# ------------------------------------------------------------------------------------------------
class _Ref:
    """Both oracles over one synthetic graph: the C DFS (fixed-length patterns) and the Python
    restatement (everything else)."""

    def __init__(self, g, simple):
        from oracle import dfs
        from tests.rmat_oracle import refdb_from_csr
        self.g = g
        self.cg = dfs.CsrGraph(g.csr[0], g.csr[1], {"uid": np.arange(g.V, dtype=np.int64), "age": g.age},
                               simple=simple)
        self._db = None
        self.bindings = None  # the C DFS's complete matches of the last expected() it answered
        self._memo = {}  # (query, cols) → (rows, bindings): the same case is checked under several modes

    @property
    def db(self):
        if self._db is None:
            from tests.rmat_oracle import refdb_from_csr
            self._db = refdb_from_csr(self.g.csr[0], self.g.csr[1], self.g.age)
        return self._db

    def expected(self, query, cols):
        key = (query, tuple(cols) if cols is not None else None)
        if key not in self._memo:
            rows = self._expected(query, cols)
            self._memo[key] = (rows, self.bindings)
        rows, self.bindings = self._memo[key]
        return rows

    def _expected(self, query, cols):
        from oracle import dfs
        self.bindings = None
        if cols is not None:
            try:
                r = dfs.run(self.cg, query, nthreads=8)
                idx = [r["aliases"].index(c) for c in cols]
                self.bindings = r["bindings"]
                return {tuple((11 << 48) | int(v) for v in row[idx]) for row in r["rows"]}
            except NotImplementedError:
                pass
        return oracle_set(oracle_rows(self.db, query), cols)


@pytest.fixture(scope="module")
def rmat10():
    import orientdb_amd as o
    g = o.GraphSnapshot.rmat(10, device=0, keep_csr=True)
    return g, _Ref(g, True)


@pytest.fixture(scope="module")
def rmat10_raw():
    """parallel edges and self loops kept (ridbag multiplicity, OSBTreeRidBag.java:292-295)"""
    import orientdb_amd as o
    g = o.GraphSnapshot.rmat(10, device=0, simple=False, keep_csr=True)
    return g, _Ref(g, False)


@pytest.fixture(scope="module")
def rmat16():
    import orientdb_amd as o
    g = o.GraphSnapshot.rmat(16, device=0, keep_csr=True)
    return g, _Ref(g, True)


RMAT_QUERIES = [
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
    ("elements", "MATCH {class:Person,as:a,where:(age = 13)}.out('Knows'){as:b} RETURN $elements", None),
    ("varlen_depth", "MATCH {class:Person,as:s,where:(uid = 5)}-Knows->{as:v, while:($depth < 3)} RETURN s, v", ["s", "v"]),
    ("varlen_where_depth", "MATCH {class:Person,as:s,where:(uid < 4)}-Knows->{as:v, while:($depth < 3), where:($depth = 2)} RETURN s, v",
     ["s", "v"]),
    ("varlen_maxdepth", "MATCH {class:Person,as:s,where:(uid = 9)}-Knows->{as:v, maxDepth: 2, where:(age < 50)} RETURN s, v", ["s", "v"]),
    ("varlen_while_prop", "MATCH {class:Person,as:s,where:(uid < 3)}-Knows->{as:v, maxDepth: 3, while:(age < 60)} RETURN s, v",
     ["s", "v"]),
    ("cartesian", "MATCH {class:Person,as:a,where:(uid < 3)},{class:Person,as:b,where:(uid > 1020)} RETURN a,b", ["a", "b"]),
    # WHERE conjuncts on the row's bindings ($matched.X op $currentMatch, OMatchPathItem.java:49-78)
    ("fof_not_me", "MATCH {class:Person,as:me,where:(age < 10)}-Knows->{}-Knows->{as:f, where:($matched.me != $currentMatch)} RETURN me, f",
     ["me", "f"]),
    ("fof_is_me", "MATCH {class:Person,as:me,where:(age < 30)}-Knows->{}-Knows->{as:f, where:($currentMatch = $matched.me)} RETURN me, f",
     ["me", "f"]),
    ("matched_and_filter", "MATCH {class:Person,as:me,where:(age < 20)}<-Knows-{as:x}-Knows->{as:f, where:($matched.me <> $currentMatch and age < 50)} RETURN me, x, f",
     ["me", "x", "f"]),
    # a bound (cycle-closing) target with a row-level conjunct: the forward check filters with it (:468-477)
    ("matched_bound", "MATCH {class:Person,as:a,where:(uid < 40)}-Knows->{as:b}-Knows->{as:c},"
                      "{as:a}-Knows->{as:c, where:($matched.b != $currentMatch and age < 70)} RETURN a, b, c",
     ["a", "b", "c"]),
    ("matched_bound_eq", "MATCH {class:Person,as:a,where:(uid < 200)}-Knows->{as:b}-Knows->{as:c},"
                         "{as:b}-Knows->{as:c, where:($currentMatch = $matched.a)} RETURN a, b, c", ["a", "b", "c"]),
    # row-level conjuncts on the outputs of a variable-length and of a multi-step item
    ("matched_varlen", "MATCH {class:Person,as:s,where:(uid < 20)}-Knows->{as:m}-Knows->{as:v, maxDepth: 2, "
                       "where:($matched.s != $currentMatch and age < 80)} RETURN s, m, v", ["s", "m", "v"]),
    ("matched_varlen_eq", "MATCH {class:Person,as:s,where:(uid < 60)}-Knows->{as:v, while:($depth < 3), "
                          "where:($matched.s = $currentMatch)} RETURN s, v", ["s", "v"]),
    ("matched_multi", "MATCH {class:Person,as:a,where:(uid < 20)}.(out('Knows').out('Knows')){as:c, "
                      "where:($matched.a <> $currentMatch)} RETURN a, c", ["a", "c"]),
    # b's WHERE declared on another occurrence of the alias: rebindFilters (P/OMatchStatement.java:185-195)
    # gives the forward hop into b the merged filter, so that hop is filtered and set-valued
    ("where_other_occurrence", "MATCH {class:Person,as:a,where:(uid < 60)}-Knows->{as:b}, {as:b,where:(age < 50)} RETURN a,b",
     ["a", "b"]),
    ("bound_candidate", "MATCH {class:Person,as:a,where:(uid = 1)}-Knows->{as:b},{class:Person,as:b,where:(uid < 600)} RETURN a,b",
     ["a", "b"]),
    # optional nodes (P/OMatchStatement.java:448-458): unmatched → the row continues with a null alias
    ("optional_free", "MATCH {class:Person,as:a,where:(uid < 80)}-Knows->{as:b, where:(age < 3), optional:true} RETURN a, b",
     ["a", "b"]),
    ("optional_bound", "MATCH {class:Person,as:a,where:(uid < 40)}-Knows->{as:c, optional:true},"
                       "{as:a}-Knows->{as:b}-Knows->{as:c, optional:true} RETURN a, b, c", ["a", "b", "c"]),
    # multi-step items .( ... ) (P/OMultiMatchPathItem.java:41-61)
    ("multi_two_hops", "MATCH {class:Person,as:a,where:(uid < 20)}.(out('Knows').out('Knows')){as:c, where:(age < 30)} RETURN a, c",
     ["a", "c"]),
    ("multi_varlen", "MATCH {class:Person,as:a,where:(uid < 6)}.(out('Knows'){where:(age < 70)}.in('Knows')){as:c, while:($depth < 2)} RETURN a, c",
     ["a", "c"]),
    ("multi_edge_pair", "MATCH {class:Person,as:a,where:(uid < 12)}.(outE('Knows').inV()){as:b, where:(age > 50)} RETURN a, b",
     ["a", "b"]),
]


DOC_QUERIES = [
    ("alias_fields", "MATCH {class:Person,as:a,where:(age < 3)}-Knows->{as:b} RETURN a.uid, b.age"),
    ("field_dedup", "MATCH {class:Person,as:a,where:(age < 10)}-Knows->{as:b} RETURN b.age as age"),
    ("expr_math", "MATCH {class:Person,as:a,where:(uid < 30)}-Knows->{as:b} RETURN a.uid * 1000 + b.age as k, a"),
    ("json", "MATCH {class:Person,as:a,where:(uid < 20)}-Knows->{as:b} RETURN {'a': a.uid, 'n': b.age + 1, 'r': b}"),
    ("out_list", "MATCH {class:Person,as:a,where:(uid < 15)} RETURN a.out('Knows').size() as d, a.out('Knows')[0-2] as f"),
    ("optional_expr", "MATCH {class:Person,as:a,where:(uid < 60)}-Knows->{as:b, where:(age < 4), optional:true} RETURN a, b.uid"),
]


DOC_QUERIES += [
    ("math_dbl", "MATCH {class:Person,as:a,where:(uid < 40)}-Knows->{as:b} RETURN b.age / 2.0 as h, b.age % 7 as m"),
    ("rid_and_const", "MATCH {class:Person,as:a,where:(uid < 25)}-Knows->{as:b} RETURN b.@rid as r, 3 as k, a.nope as z"),
    ("int_div", "MATCH {class:Person,as:a,where:(uid < 25)}-Knows->{as:b} RETURN (a.uid + 7) / 3 as q, -a.uid as n"),
    # Java integer arithmetic on negatives: / truncates toward zero, % keeps the dividend's sign
    ("neg_div_mod", "MATCH {class:Person,as:a,where:(uid < 40)}-Knows->{as:b} RETURN (a.uid - 20) / 7 as q, (a.uid - 20) % 7 as m"),
]


@pytest.mark.parametrize("devproj", ["device", "host"])
@pytest.mark.parametrize("q", DOC_QUERIES, ids=[q[0] for q in DOC_QUERIES])
def test_rmat_documents(rmat10, q, devproj, monkeypatch):
    """RETURN expressions / JSON (addResult :698-719, jsonToDoc :791-806): documents equal by content —
    scalar items evaluated and de-duplicated on the device (projdev.hip), or every item through the host
    evaluator (OMX_DEVPROJ=0, and always for JSON, lists and methods)."""
    import orientdb_amd as o
    monkeypatch.setenv("OMX_DEVPROJ", "1" if devproj == "device" else "0")
    g, ref = rmat10
    want = oracle_rows(ref.db, q[1])
    rs = o.OMatchStatement(q[1]).execute(g)
    assert rs.info["documents"] == 1
    assert len(rs) == len(want)
    if "[0-2]" in q[1]:  # list order = ridbag order (unpinned): compare as multisets of lengths and sizes
        assert sorted((d["d"], len(d["f"])) for d in rs) == sorted((d["d"], len(d["f"])) for d in want)
        return
    assert doc_set(rs) == doc_set(want)


@pytest.mark.parametrize("devproj", ["1", "0"])
def test_return_division_by_zero_fails(rmat10, devproj, monkeypatch):
    """An integer division by zero in a RETURN item fails the execution on both evaluators."""
    import orientdb_amd as o
    monkeypatch.setenv("OMX_DEVPROJ", devproj)
    g, _ = rmat10
    with pytest.raises(o.OmxExecutionError):
        o.OMatchStatement("MATCH {class:Person,as:a,where:(uid < 5)} RETURN a.uid / 0 as x").execute(g)


@pytest.mark.parametrize("devproj", ["1", "0"])
def test_return_division_by_zero_past_limit(rmat10, devproj, monkeypatch):
    """LIMIT stops the projection at the limit-th distinct document (OMatchStatement.addSingleResult
    :737-750), so a division by zero in a later row is never evaluated: the rows of one alias come in
    ascending vertex order, the zero divisor sits on the last root, and LIMIT 1 returns the first root's
    document on both evaluators (the device one hands LIMIT to the host, which stops early); without the
    LIMIT both fail."""
    import orientdb_amd as o
    from oracle.match_ref import MatchOracle
    monkeypatch.setenv("OMX_DEVPROJ", devproj)
    g, ref = rmat10
    rp = g.csr[0].astype(np.int64)
    roots = [v for v in range(30) if rp[v + 1] > rp[v]]
    last = roots[-1]
    q = "MATCH {class:Person,as:a,where:(uid < 30)}-Knows->{as:b} RETURN 1000 / (a.uid - %d) as x" % last
    rs = o.OMatchStatement(q + " LIMIT 1").execute(g)
    assert len(rs) == 1
    want = MatchOracle(ref.db, q + " LIMIT 1").execute()
    assert doc_set(rs) == doc_set(want)
    with pytest.raises(o.OmxExecutionError):
        o.OMatchStatement(q).execute(g)


def test_optional_null_reached_again_raises(rmat10):
    """A null optional alias reached again by a non-empty traversal is the reference's
    NullPointerException (matched.get(alias).getIdentity(), P/OMatchStatement.java:468): an execution error."""
    import orientdb_amd as o
    from oracle.match_ref import OracleError
    g, ref = rmat10
    q = ("MATCH {class:Person,as:a,where:(uid < 40)}-Knows->{as:b}-Knows->{as:c, where:(age < 30), optional:true},"
         "{as:a}-Knows->{as:c, optional:true} RETURN a, b, c")
    with pytest.raises(OracleError):
        oracle_rows(ref.db, q)
    with pytest.raises(o.OmxExecutionError):
        o.OMatchStatement(q).execute(g)


def _parity(g, ref, query, cols, **kw):
    import orientdb_amd as o
    want = ref.expected(query, cols)
    rs = o.OMatchStatement(query).execute(g, **kw)
    assert rs.info["n_rows"] == len(want)
    assert gpu_set(rs, cols if cols and rs.columns[0] not in ("$elements", "$pathElements") else None) == want
    if ref.bindings is not None and "LIMIT" not in query.upper():
        # complete matches before the de-duplication: a set-valued hop binds a repeated neighbour once
        # (P/OMatchPathItem.java:61,71-78), reverse hops and hops without a WHERE once per edge
        assert rs.info["bindings"] == ref.bindings
    return rs


@pytest.mark.parametrize("q", RMAT_QUERIES, ids=[q[0] for q in RMAT_QUERIES])
def test_rmat_parity(rmat10, q):
    g, ref = rmat10
    _parity(g, ref, q[1], q[2])


@pytest.mark.parametrize("q", RMAT_QUERIES, ids=[q[0] for q in RMAT_QUERIES])
def test_rmat_parity_all_rows_chunked(rmat10, q, monkeypatch):
    """Same cases with every row of degree ≥ 2 routed through the chunked (heavy-row) kernel."""
    monkeypatch.setenv("OMX_HEAVY_DEG", "2")
    g, ref = rmat10
    _parity(g, ref, q[1], q[2])


CHUNK_IDS = ("c2_both_ends", "c1_fof", "c1_abc", "both_dir", "three_hop", "paths", "varlen_depth", "cartesian",
             "optional_free", "multi_two_hops")


@pytest.mark.parametrize("chunk", ["256", "512", "2048"])
@pytest.mark.parametrize("q", [q for q in RMAT_QUERIES if q[0] in CHUNK_IDS], ids=lambda q: q[0])
def test_rmat_parity_dense_chunk_windows(rmat10, q, chunk, monkeypatch):
    """Unfiltered written hops with every row of degree ≥ 2 cut into 256-, 512- or 2048-entry aligned
    chunk windows (k_expand_heavy with 4 / 8 / 32 slots), factorized hops forced so their row emission
    takes it."""
    monkeypatch.setenv("OMX_HEAVY_DEG_UNFILTERED", "2")
    monkeypatch.setenv("OMX_UNF_CHUNK", chunk)
    monkeypatch.setenv("OMX_FACTOR", "force")
    g, ref = rmat10
    _parity(g, ref, q[1], q[2])


MARK_QUERIES = [
    ("fof", "MATCH {class:Person}-Knows->{}-Knows->{as:fof} RETURN fof", ["fof"]),
    ("fof_window", "MATCH {class:Person,as:a,where:(age < 20)}-Knows->{as:b}-Knows->{as:c} RETURN c", ["c"]),
    ("both_dir", "MATCH {class:Person,as:a,where:(age < 10)}-Knows-{as:b}-Knows-{as:c} RETURN c", ["c"]),
    ("in_dir", "MATCH {class:Person,as:a,where:(age < 30)}<-Knows-{as:b}<-Knows-{as:c} RETURN c", ["c"]),
    ("three_hop", "MATCH {class:Person,as:a,where:(uid < 8)}-Knows->{}-Knows->{}-Knows->{as:d} RETURN d", ["d"]),
]


MARK_CASES = [(q, h, f) for q in MARK_QUERIES for h in ("default", "all_heavy") for f in ("force", "0")
              if not (q[0] == "fof" and h == "all_heavy")]  # (fof: every Person a root, the oracle's slowest)


@pytest.mark.parametrize("q,heavy,factor", MARK_CASES, ids=lambda x: x[0] if isinstance(x, tuple) else str(x))
def test_rmat_parity_marked_last_hop(rmat10, rmat10_raw, q, heavy, factor, monkeypatch):
    """A plan returning only its last alias, de-duplicated: the last hop marks the distinct neighbours
    as it reads them (Executor::expand_mark) — same rows, bindings and E_t as writing the rows and
    marking them in the projection (OMX_MARK_FUSE=0), on the simple graph and the multigraph."""
    import orientdb_amd as o
    if heavy == "all_heavy":
        monkeypatch.setenv("OMX_HEAVY_DEG", "2")
    # force: each distinct source's neighbours marked once (the rows repeat their sources); 0: every row's
    monkeypatch.setenv("OMX_FACTOR", factor)
    for g, ref in (rmat10, rmat10_raw):
        monkeypatch.setenv("OMX_MARK_FUSE", "1")
        rs = _parity(g, ref, q[1], q[2])
        monkeypatch.setenv("OMX_MARK_FUSE", "0")
        plain = o.OMatchStatement(q[1]).execute(g, documents=False)
        assert rs.info["bindings"] == plain.info["bindings"]
        assert rs.info["edges_traversed"] == plain.info["edges_traversed"]
        assert rs.info["n_rows"] == plain.info["n_rows"]


SLICED_IDS = ("c2_both_ends", "in_dir", "both_dir", "three_hop", "triangle_filtered", "matches", "varlen_maxdepth",
              "two_cols_dedup")


@pytest.mark.parametrize("q", [q for q in RMAT_QUERIES if q[0] in SLICED_IDS], ids=lambda q: q[0])
def test_rmat_parity_sliced(rmat10, q, monkeypatch):
    """Filtered hops through the LDS-sliced heavy kernel with 64-vertex bitmap slices (V = 1024 →
    16 slices), so every heavy row's adjacency is cut at many slice boundaries."""
    monkeypatch.setenv("OMX_HEAVY_DEG", "2")
    monkeypatch.setenv("OMX_SLICE_SHIFT", "6")
    g, ref = rmat10
    _parity(g, ref, q[1], q[2])
    c = __import__("orientdb_amd").OMatchStatement(q[1]).execute(g, mode=__import__("orientdb_amd").OMX_MODE_COUNT)
    assert c.info["edges_traversed"] >= 0


@pytest.mark.parametrize("light_sliced", ["1", "0"], ids=["light_sliced", "light_merge_path"])
@pytest.mark.parametrize("q", [q for q in RMAT_QUERIES if q[0] in SLICED_IDS], ids=lambda q: q[0])
def test_rmat_parity_sliced_light_rows(rmat10, q, light_sliced, monkeypatch):
    """Rows of degree < 16 of a sliced hop through the LDS-sliced light kernel (16 slices of 64
    vertices: each light row is cut into pieces, 64 rows' pieces packed per slot group), and through
    the merge-path kernel."""
    import orientdb_amd as o
    monkeypatch.setenv("OMX_HEAVY_DEG", "16")
    monkeypatch.setenv("OMX_SLICE_SHIFT", "6")
    monkeypatch.setenv("OMX_LIGHT_SLICED", light_sliced)
    g, ref = rmat10
    _parity(g, ref, q[1], q[2])
    m = o.OMatchStatement(q[1]).execute(g)
    c = o.OMatchStatement(q[1]).execute(g, mode=o.OMX_MODE_COUNT)
    assert c.info["n_rows"] == m.info["n_rows"]


@pytest.mark.parametrize("q", [q for q in RMAT_QUERIES if q[0] in SLICED_IDS], ids=lambda q: q[0])
def test_rmat_parity_l2_probe_heavy(rmat10, q, monkeypatch):
    """The same cases through the L2-probe heavy kernel (slicing disabled)."""
    monkeypatch.setenv("OMX_HEAVY_DEG", "2")
    monkeypatch.setenv("OMX_SLICED", "0")
    g, ref = rmat10
    _parity(g, ref, q[1], q[2])


FACTOR_IDS = ("c2_both_ends", "c1_abc", "two_cols_dedup", "in_dir", "both_dir", "three_hop", "triangle_filtered", "matches",
              "paths", "elements", "fof_not_me", "matched_and_filter", "optional_free", "bound_candidate")


@pytest.mark.parametrize("graph", ["simple", "multigraph"])
@pytest.mark.parametrize("q", [q for q in RMAT_QUERIES if q[0] in FACTOR_IDS], ids=lambda q: q[0])
def test_rmat_parity_factorized(rmat10, rmat10_raw, q, graph, monkeypatch):
    """Every filtered hop through the factorized expansion (distinct sources → filtered lists → rows
    over the lists, Executor::expand_factorized): same rows, same E_t and bindings as the direct
    expansion — on the simple graph and on the multigraph, whose parallel edges repeat a neighbour in a
    source's list (ridbag multiplicity, OSBTreeRidBag.java:292-295) through the distinct-source grouping.
    The rows are written by the output-tiled emission at any size (OMX_FEMIT=force)."""
    import orientdb_amd as o
    g, ref = rmat10 if graph == "simple" else rmat10_raw
    monkeypatch.setenv("OMX_FEMIT", "force")
    monkeypatch.setenv("OMX_FACTOR", "0")
    direct = o.OMatchStatement(q[1]).execute(g, documents=False)
    monkeypatch.setenv("OMX_FACTOR", "force")
    rs = _parity(g, ref, q[1], q[2])
    assert direct.info["factorized_hops"] == 0
    assert rs.info["edges_traversed"] == direct.info["edges_traversed"]
    assert rs.info["bindings"] == direct.info["bindings"]


EMIT_CASES = [(q, g, e) for q in RMAT_QUERIES if q[0] in FACTOR_IDS for g in ("simple", "multigraph") for e in ("binned",)] + \
    [(q, "multigraph", e) for q in RMAT_QUERIES if q[0] in ("c2_both_ends", "in_dir", "three_hop", "paths", "matched_and_filter")
     for e in ("slow", "grp64")]


@pytest.mark.parametrize("q,graph,emit", EMIT_CASES, ids=lambda x: x[0] if isinstance(x, tuple) else str(x))
def test_rmat_parity_factorized_emission(rmat10, rmat10_raw, q, graph, emit, monkeypatch):
    """The factorized hop's rows written the other ways (the default — rows grouped by source, output
    tiles of k_femit_w — is covered by test_rmat_parity_factorized): binned = the generic unfiltered
    expansion over the lists (OMX_FEMIT=0); slow = every output tile through k_femit_slow (a search of
    the row offsets per output row); grp64 = the lists grouped with 64-bit counters and cursors
    (OMX_GRP32=0, the path of lists of 2^32 or more entries). Same rows, E_t and bindings as the direct
    expansion (P/OMatchStatement.java:491-497 per row)."""
    import orientdb_amd as o
    g, ref = rmat10 if graph == "simple" else rmat10_raw
    monkeypatch.setenv("OMX_FACTOR", "0")
    direct = o.OMatchStatement(q[1]).execute(g, documents=False)
    monkeypatch.setenv("OMX_FACTOR", "force")
    monkeypatch.setenv("OMX_FEMIT", "0" if emit == "binned" else "force")
    monkeypatch.setenv("OMX_FEMIT_SLOW", "1" if emit == "slow" else "0")
    monkeypatch.setenv("OMX_GRP32", "0" if emit == "grp64" else "1")
    rs = _parity(g, ref, q[1], q[2])
    assert rs.info["edges_traversed"] == direct.info["edges_traversed"]
    assert rs.info["bindings"] == direct.info["bindings"]


@pytest.mark.parametrize("slow", ["0", "1"])
def test_factorized_emission_many_tiles_rmat16(rmat16, slow, monkeypatch):
    """Output tiles of the factorized emission across many tiles (RMAT-16 2-hop with WHERE on both ends:
    rows spanning tile boundaries, runs of short lists in one tile, a partial last tile): rows and digest
    equal with the emission through the generic expansion."""
    import orientdb_amd as o
    g = rmat16[0]
    q = "MATCH {class:Person,as:a,where:(age < 20)}-Knows->{as:b}-Knows->{as:c,where:(age >= 60)} RETURN a,b,c"
    monkeypatch.setenv("OMX_FACTOR", "force")
    monkeypatch.setenv("OMX_FEMIT", "0")
    fl = o.OMX_FLAG_KEEP_DEVICE | o.OMX_FLAG_DIGEST
    base = o.OMatchStatement(q).execute(g, documents=False, flags=fl)
    monkeypatch.setenv("OMX_FEMIT", "force")
    monkeypatch.setenv("OMX_FEMIT_SLOW", slow)
    rs = o.OMatchStatement(q).execute(g, documents=False, flags=fl)
    assert rs.info["factorized_hops"] >= 1 and rs.info["n_rows"] > 100000
    assert rs.info["n_rows"] == base.info["n_rows"] and rs.info["digest"] == base.info["digest"]
    assert rs.info["edges_traversed"] == base.info["edges_traversed"]


@pytest.mark.parametrize("lists", ["flists", "sliced"])
@pytest.mark.parametrize("graph", ["simple", "multigraph"])
@pytest.mark.parametrize("q", [q for q in RMAT_QUERIES if q[0] in FACTOR_IDS], ids=lambda q: q[0])
def test_factorized_lists_paths(rmat10, rmat10_raw, q, graph, lists, monkeypatch):
    """The distinct sources' filtered lists through the hub-annotated col (factor.hip k_flists: LDS table
    per tile, or every tile's sources found by binary search) and through the sliced expansion + grouping
    (OMX_FLISTS=0): the oracle's rows, bindings and E_t on every factorized hop, both emissions. (On the
    multigraph a set-valued hop keeps the sliced path: its lists are made distinct there.)"""
    import orientdb_amd as o
    g, ref = rmat10 if graph == "simple" else rmat10_raw
    monkeypatch.setenv("OMX_FACTOR", "force")
    monkeypatch.setenv("OMX_FLISTS", {"flists": "1", "sliced": "0"}[lists])
    for emit in ("force", "0"):
        monkeypatch.setenv("OMX_FEMIT", emit)
        rs = _parity(g, ref, q[1], q[2])
        if q[0] in ("c2_both_ends", "in_dir", "three_hop"):
            assert rs.info["factorized_hops"] >= 1


def test_factorized_lists_rmat16_digest(rmat16, monkeypatch):
    """k_flists at RMAT-16 (thousands of tiles, hubs of degree ~10^3 spanning many tiles: the survivors of
    a source continuing over tiles are placed through the tiles' last-source counts): rows, E_t, bindings
    and digest equal the sliced path's and dfs_ref.c's."""
    import orientdb_amd as o
    from oracle import dfs
    g, ref = rmat16
    q = "MATCH {class:Person,as:a,where:(age < 3)}-Knows->{as:b}-Knows->{as:c,where:(age >= 80)} RETURN a,b,c"
    want = dfs.run(ref.cg, q, nthreads=8, emit=False, digest=["a", "b", "c"])
    monkeypatch.setenv("OMX_FACTOR", "force")
    out = {}
    for lists in ("1", "0"):
        monkeypatch.setenv("OMX_FLISTS", lists)
        rs = o.OMatchStatement(q).execute(g, flags=o.OMX_FLAG_KEEP_DEVICE | o.OMX_FLAG_DIGEST, documents=False)
        out[lists] = (rs.info["n_rows"], rs.info["edges_traversed"], rs.info["bindings"], rs.info["digest"])
    assert out["1"] == out["0"]
    assert out["1"][2] == want["bindings"] and out["1"][1] == want["edges"] and out["1"][3] == want["digest"]


@pytest.mark.parametrize("every", [1, 7, 300])
def test_factorized_lists_sparse_sources(every, monkeypatch):
    """k_flists when most distinct sources have no out-edge: root 0 reaches b = 1 … 3000, and only every
    `every`-th b has out-edges (to 3001 + (b mod 97) and 3001 + (b mod 89)). Sources without chunks still
    count in a tile's source range, so a tile spans more than its 128 chunk slots' sources and goes to
    k_flist_wide (every = 7, 300); rows equal the brute-force enumeration on both lists paths."""
    import orientdb_amd as o
    nb, V = 3000, 3200
    out = {0: list(range(1, nb + 1))}
    for b in range(1, nb + 1):
        if b % every == 0:
            out[b] = sorted({3001 + b % 97, 3001 + b % 89})
    rp = np.zeros(V + 1, np.uint64)
    rp[1:] = np.cumsum([len(out.get(v, [])) for v in range(V)])
    col = np.array([t for v in range(V) for t in out.get(v, [])], np.uint32)
    g = o.GraphSnapshot.person_knows(rp, col, seed=3, device=0, keep_csr=True)
    q = "MATCH {class:Person,as:a,where:(uid = 0)}-Knows->{as:b}-Knows->{as:c,where:(age >= 0)} RETURN a,b,c"
    want = sorted((0, b, c) for b in out[0] for c in out.get(b, []))
    monkeypatch.setenv("OMX_FACTOR", "force")
    for lists in ("1", "0"):
        monkeypatch.setenv("OMX_FLISTS", lists)
        rs = o.OMatchStatement(q).execute(g, documents=False)
        got = sorted(tuple(int(x) & ((1 << 48) - 1) for x in row) for row in rs.rows)
        assert got == want, lists
        assert rs.info["factorized_hops"] >= 1
    g.close()


@pytest.mark.parametrize("case", ["m1_shape_rmat16", "deferred_tiles", "multigraph_set_valued"])
def test_factorized_lists_poisoned_pool(rmat16, rmat10_raw, case, monkeypatch):
    """The factorized hop's scratch under OMX_POOL_POISON=1: every device buffer the pool hands out is
    0xFF-filled first, so a kernel that reads a word it never wrote (a zero-survivor tile's scratch slot
    used as a hub index — the illegal access of round 5's uncommitted k_flist_copy variant, DESIGN.md
    "Round 5: the k_flist_copy fault") reads 0xFFFFFFFF instead of a lucky zero and faults or differs.
    Cases: M1's query shape at RMAT-16 (k_flists + k_femit_w), tiles spanning more sources than their
    slots (k_flist_wide, the deferred tiles), and the multigraph's set-valued hop (lists made distinct)."""
    import orientdb_amd as o
    from oracle import dfs
    monkeypatch.setenv("OMX_POOL_POISON", "1")
    monkeypatch.setenv("OMX_FACTOR", "force")
    monkeypatch.setenv("OMX_FEMIT", "force")
    if case == "m1_shape_rmat16":
        g, ref = rmat16
        q = "MATCH {class:Person,as:a,where:(age < 3)}-Knows->{as:b}-Knows->{as:c,where:(age >= 80)} RETURN a,b,c"
        want = dfs.run(ref.cg, q, nthreads=8, emit=False, digest=["a", "b", "c"])
        rs = o.OMatchStatement(q).execute(g, flags=o.OMX_FLAG_KEEP_DEVICE | o.OMX_FLAG_DIGEST, documents=False)
        assert rs.info["factorized_hops"] >= 1
        assert (rs.info["n_rows"], rs.info["edges_traversed"], rs.info["digest"]) == \
            (want["bindings"], want["edges"], want["digest"])
        d = o.OMatchStatement(q).execute(g, documents=False)  # the rows handed to the host, poisoned staging
        assert dfs.row_digest(d.rows) == want["digest"]
    elif case == "deferred_tiles":
        nb, V = 3000, 3200
        out = {0: list(range(1, nb + 1))}
        for b in range(7, nb + 1, 7):
            out[b] = sorted({3001 + b % 97, 3001 + b % 89})
        rp = np.zeros(V + 1, np.uint64)
        rp[1:] = np.cumsum([len(out.get(v, [])) for v in range(V)])
        col = np.array([t for v in range(V) for t in out.get(v, [])], np.uint32)
        g = o.GraphSnapshot.person_knows(rp, col, seed=3, device=0, keep_csr=True)
        q = "MATCH {class:Person,as:a,where:(uid = 0)}-Knows->{as:b}-Knows->{as:c,where:(age >= 0)} RETURN a,b,c"
        rs = o.OMatchStatement(q).execute(g, documents=False)
        got = sorted(tuple(int(x) & ((1 << 48) - 1) for x in row) for row in rs.rows)
        assert got == sorted((0, b, c) for b in out[0] for c in out.get(b, []))
        g.close()
    else:
        g, ref = rmat10_raw
        q = next(x for x in RMAT_QUERIES if x[0] == "c2_both_ends")
        for lists in ("1", "0"):
            monkeypatch.setenv("OMX_FLISTS", lists)
            _parity(g, ref, q[1], q[2])


SEMI_QUERIES = [
    ("ab_of_abc", "MATCH {class:Person,as:a,where:(age < 5)}-Knows->{as:b}-Knows->{as:c,where:(age >= 90)} RETURN a, b",
     ["a", "b"]),
    ("expr_of_abc", "MATCH {class:Person,as:a,where:(age < 5)}-Knows->{as:b}-Knows->{as:c,where:(age >= 90)} RETURN a.uid, b.age",
     None),
    ("a_of_abc", "MATCH {class:Person,as:a,where:(age < 20)}-Knows->{as:b}-Knows->{as:c,where:(age > 50)} RETURN a", ["a"]),
    ("three_hop_abc", "MATCH {class:Person,as:a,where:(uid < 8)}-Knows->{as:b}-Knows->{as:c}-Knows->{as:d,where:(age<10)} RETURN a, b, c",
     ["a", "b", "c"]),
]


@pytest.mark.parametrize("graph", ["simple", "multigraph"])
@pytest.mark.parametrize("q", SEMI_QUERIES, ids=[q[0] for q in SEMI_QUERIES])
def test_semi_join_last_hop(rmat10, rmat10_raw, q, graph, monkeypatch):
    """A factorized last hop whose new alias the projection never reads is a semi-join (the rows whose
    source has a non-empty filtered list; no row per target is written): the same documents / rows as
    the oracle and as writing every row (OMX_SEMI=0), the same E_t and bindings (Σ |L(b)|, parallel edges
    included)."""
    import orientdb_amd as o
    g, ref = rmat10 if graph == "simple" else rmat10_raw
    monkeypatch.setenv("OMX_FACTOR", "force")
    monkeypatch.setenv("OMX_SEMI", "0")
    full = o.OMatchStatement(q[1]).execute(g, documents=q[2] is None)
    monkeypatch.setenv("OMX_SEMI", "1")
    if q[2] is not None:
        rs = _parity(g, ref, q[1], q[2])
    else:
        rs = o.OMatchStatement(q[1]).execute(g)
        assert doc_set(rs) == doc_set(oracle_rows(ref.db, q[1]))
        assert doc_set(rs) == doc_set(full)
    assert rs.info["n_rows"] == full.info["n_rows"]
    assert rs.info["edges_traversed"] == full.info["edges_traversed"]
    assert rs.info["bindings"] == full.info["bindings"]


@pytest.mark.parametrize("simple", [True, False], ids=["simple", "multigraph"])
def test_factorized_auto_threshold_rmat14(simple):
    """The factorized expansion as the planner picks it by itself (≥ 4096 rows whose sources repeat ≥ 4×,
    exec.hip expand_factorized): RMAT-14 2-hop with the WHERE on both ends, on the simple graph and the
    multigraph (parallel edges: a neighbour repeated in a source's list is one row per edge,
    OSBTreeRidBag.java:292-295). The device reports the hop as factorized; rows, E_t and bindings equal
    the DFS oracle's and the direct expansion's."""
    import orientdb_amd as o
    from oracle import dfs
    g = o.GraphSnapshot.rmat(14, device=0, simple=simple, keep_csr=True)
    q = "MATCH {class:Person,as:a,where:(age < 5)}-Knows->{as:b}-Knows->{as:c,where:(age >= 90)} RETURN a,b,c"
    cg = dfs.CsrGraph(g.csr[0], g.csr[1], {"uid": np.arange(g.V, dtype=np.int64), "age": g.age}, simple=simple)
    ref = dfs.run(cg, q, nthreads=8)
    rs = o.OMatchStatement(q).execute(g, documents=False)
    assert rs.info["factorized_hops"] >= 1
    got = {tuple(int(x) & ((1 << 48) - 1) for x in row) for row in rs.rows}
    want = {tuple(int(v) for v in row) for row in ref["rows"]}
    assert got == want and rs.info["n_rows"] == len(want)
    assert rs.info["edges_traversed"] == ref["edges"]
    # (multigraph: a forward hop into a node with a WHERE returns a HashSet in the reference
    # (OMatchPathItem.java:61,71-78), so a neighbour reached over parallel edges binds once; the device
    # makes each source's filtered list distinct, Step::distinct_nb, while E_t still counts every edge)
    assert rs.info["bindings"] == ref["bindings"]
    import os
    os.environ["OMX_FACTOR"] = "0"
    try:
        direct = o.OMatchStatement(q).execute(g, documents=False)
    finally:
        del os.environ["OMX_FACTOR"]
    assert direct.info["factorized_hops"] == 0
    assert direct.info["edges_traversed"] == rs.info["edges_traversed"]
    assert direct.info["bindings"] == rs.info["bindings"]
    g.close()


@pytest.mark.parametrize("q", [q for q in RMAT_QUERIES if q[0] in ("c2_both_ends", "in_dir", "three_hop", "matches")],
                         ids=lambda q: q[0])
def test_rmat_parity_short_arena_rerun(rmat10, q, monkeypatch):
    """Sliced hops size their output arenas from the target bitmap's density; with the margin at 0 the
    estimate is short, the kernels count the rows they could not write, and the hop re-runs with the
    exact bound (Executor::expand_core) — same rows."""
    monkeypatch.setenv("OMX_HEAVY_DEG", "2")
    monkeypatch.setenv("OMX_SLICE_SHIFT", "6")
    monkeypatch.setenv("OMX_ARENA_MARGIN", "0")
    g, ref = rmat10
    _parity(g, ref, q[1], q[2])


def test_sliced_count_mode_and_segments(rmat10, monkeypatch):
    """Count mode and the KEEP_DEVICE block-segmented result of the sliced kernel agree with the
    materialized rows."""
    import orientdb_amd as o
    monkeypatch.setenv("OMX_HEAVY_DEG", "2")
    monkeypatch.setenv("OMX_SLICE_SHIFT", "7")
    g, _ = rmat10
    q = RMAT_QUERIES[0][1]
    m = o.OMatchStatement(q).execute(g)
    c = o.OMatchStatement(q).execute(g, mode=o.OMX_MODE_COUNT)
    k = o.OMatchStatement(q).execute(g, flags=o.OMX_FLAG_KEEP_DEVICE)
    assert c.info["n_rows"] == m.info["n_rows"] == k.info["n_rows"] == c.info["bindings"] > 0
    assert c.info["edges_traversed"] == m.info["edges_traversed"] == k.info["edges_traversed"]


def test_keep_device_segmented_result(rmat10):
    """KEEP_DEVICE leaves the last filtered expansion block-segmented in HBM; row and edge counts
    equal the materialized (compacted) run."""
    import orientdb_amd as o
    g, _ = rmat10
    for q in (RMAT_QUERIES[0][1], RMAT_QUERIES[2][1]):
        m = o.OMatchStatement(q).execute(g)
        k = o.OMatchStatement(q).execute(g, flags=o.OMX_FLAG_KEEP_DEVICE)
        assert k.rows.shape[0] == 0
        assert (k.info["n_rows"], k.info["edges_traversed"], k.info["bindings"]) == \
               (m.info["n_rows"], m.info["edges_traversed"], m.info["bindings"])


@pytest.mark.parametrize("q", [q for q in RMAT_QUERIES if q[0] in ("c2_both_ends", "c1_fof", "both_dir", "triangle",
                                                                    "varlen_depth", "three_hop",
                                                                    "where_other_occurrence")],
                         ids=lambda q: q[0])
def test_rmat_parity_multigraph(rmat10_raw, q):
    g, ref = rmat10_raw
    _parity(g, ref, q[1], q[2])


RMAT16 = [  # (C4 at full size: test_gpu_triangle.py's SF10 runs against dfs_ref.c)
    ("c1_fof_sampled", "MATCH {class:Person,as:a,where:(uid < 512)}-Knows->{}-Knows->{as:fof} RETURN fof", ["fof"]),
    ("c2_both_ends", "MATCH {class:Person,as:a,where:(age < 1)}-Knows->{as:b}-Knows->{as:c,where:(age >= 90)} RETURN a,b,c",
     ["a", "b", "c"]),
]


@pytest.mark.slow
@pytest.mark.parametrize("q", RMAT16, ids=[q[0] for q in RMAT16])
def test_rmat16_parity(rmat16, q):
    """configs[0] scale (RMAT-16, the reference's CPU-runnable case) against the C oracle."""
    g, ref = rmat16
    _parity(g, ref, q[1], q[2])


@pytest.mark.slow
@pytest.mark.parametrize("q", RMAT16[1:], ids=[q[0] for q in RMAT16[1:]])
def test_rmat16_parity_sliced(rmat16, q, monkeypatch):
    """RMAT-16 through the sliced kernel cut into 16 slices of 4096 vertices, rows of degree ≥ 64."""
    monkeypatch.setenv("OMX_HEAVY_DEG", "64")
    monkeypatch.setenv("OMX_SLICE_SHIFT", "12")
    g, ref = rmat16
    _parity(g, ref, q[1], q[2])


def test_root_shards_partition_the_result(rmat10):
    """Multi-GPU partition: roots v with v % world == rank; the union over ranks is the result."""
    import orientdb_amd as o
    g, _ = rmat10
    q = RMAT_QUERIES[0][1]
    full = gpu_set(o.OMatchStatement(q).execute(g))
    parts = [gpu_set(o.OMatchStatement(q).execute(g, shard=(r, 4))) for r in range(4)]
    assert set().union(*parts) == full
    assert sum(len(p) for p in parts) == len(full)


@pytest.mark.parametrize("fuse", ["1", "0"], ids=["fof2", "general"])
def test_root_shards_fof(rmat10, fuse, monkeypatch):
    """configs[0]'s shape under root shards (the replicated multi-GPU bench's C1): k_fof2_a's shard filter
    (a.rank / a.world), or the general root → hop → marked hop path (OMX_MARK_FUSE=0). A fof may be reached
    from roots of several shards, so the shards' sets overlap: their union is the full set, and their
    bindings and E_t add up to the full run's."""
    import orientdb_amd as o
    monkeypatch.setenv("OMX_MARK_FUSE", fuse)
    g, ref = rmat10
    q = next(x for x in RMAT_QUERIES if x[0] == "c1_fof")
    full = _parity(g, ref, q[1], q[2])
    parts = [o.OMatchStatement(q[1]).execute(g, shard=(r, 3), documents=False) for r in range(3)]
    assert set().union(*(gpu_set(p, q[2]) for p in parts)) == gpu_set(full, q[2])
    assert sum(p.info["bindings"] for p in parts) == full.info["bindings"]
    assert sum(p.info["edges_traversed"] for p in parts) == full.info["edges_traversed"]


def test_count_mode_matches_materialize(rmat10):
    import orientdb_amd as o
    g, _ = rmat10
    q = RMAT_QUERIES[0][1]
    m = o.OMatchStatement(q).execute(g)
    c = o.OMatchStatement(q).execute(g, mode=o.OMX_MODE_COUNT)
    assert c.info["n_rows"] == m.info["n_rows"] == c.info["bindings"]
    assert c.info["edges_traversed"] == m.info["edges_traversed"]


def test_kernel_timing_reports_expand(rmat10):
    import orientdb_amd as o
    g, _ = rmat10
    rs = o.OMatchStatement(RMAT_QUERIES[0][1]).execute(g, flags=o.OMX_FLAG_KERNEL_TIMING)
    names = {k["name"] for k in rs.kernel_stats}
    assert any(n.startswith("k_expand_") for n in names) and "k_eval_bitmap" in names


def test_empty_and_edge_cases(rmat10):
    import orientdb_amd as o
    g, ref = rmat10
    db = ref.db
    # no root passes the filter → empty
    assert o.OMatchStatement("MATCH {class:Person,as:a,where:(age > 1000)}-Knows->{as:b} RETURN a,b").execute(g).info["n_rows"] == 0
    # unknown edge label → no neighbours
    assert o.OMatchStatement("MATCH {class:Person,as:a,where:(uid = 1)}-Nope->{as:b} RETURN a,b").execute(g).info["n_rows"] == 0
    # parameters
    rs = o.OMatchStatement("MATCH {class:Person,as:a,where:(uid = ?)}-Knows->{as:b} RETURN a,b").execute(g, 7)
    ref = oracle_rows(db, "MATCH {class:Person,as:a,where:(uid = 7)}-Knows->{as:b} RETURN a,b")
    assert gpu_set(rs) == oracle_set(ref, ["a", "b"])
    # LIMIT: count only
    rs = o.OMatchStatement("MATCH {class:Person,as:a}-Knows->{as:b} RETURN a,b LIMIT 5").execute(g)
    assert rs.info["n_rows"] == 5
