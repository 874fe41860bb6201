"""Cyclic patterns (configs[3]): the expansion that binds the last alias of a cycle and the
check that closes it run fused as an intersection of two sorted adjacency lists, so wedges are never
materialised: rows whose lists have comparable lengths through the merge path (isect.hip k_isect_merge),
the others by binary search of the shorter list into the longer one inside the expansion kernels.
Parity: identical rows to the oracle and to the unfused expand + check path, and the same traversed-edge
count (the fused kernels add Σ |N(closing vertex)| over the wedges, as the check would), with the merge
chosen by its length-ratio rule (merge), forced on every row that fits a tile (merge_force), and off
(probe: every row binary-searches).
"""
import numpy as np
import pytest

from tests.test_gpu_parity import _parity, gpu_set, rmat10, rmat10_raw, rmat16  # noqa: F401  (fixtures)

pytestmark = pytest.mark.gpu

CYCLES = [
    ("triangle", "MATCH {class:Person,as:a}-Knows->{as:b}-Knows->{as:c}-Knows->{as:a} RETURN a,b,c"),
    ("triangle_where_c", "MATCH {class:Person,as:a,where:(age < 30)}-Knows->{as:b}-Knows->{as:c,where:(age > 20)}-Knows->{as:a} RETURN a,b,c"),
    ("triangle_where_b", "MATCH {class:Person,as:a}-Knows->{as:b,where:(age < 50)}-Knows->{as:c}-Knows->{as:a} RETURN a,b,c"),
    ("triangle_in", "MATCH {class:Person,as:a,where:(uid < 300)}<-Knows-{as:b}<-Knows-{as:c}<-Knows-{as:a} RETURN a,b,c"),
    ("triangle_both", "MATCH {class:Person,as:a,where:(uid < 40)}-Knows-{as:b}-Knows-{as:c}-Knows-{as:a} RETURN a,b,c"),
    ("square", "MATCH {class:Person,as:a,where:(uid < 25)}-Knows->{as:b}-Knows->{as:c}-Knows->{as:d}-Knows->{as:a} RETURN a,b,c,d"),
    ("triangle_project", "MATCH {class:Person,as:a}-Knows->{as:b}-Knows->{as:c}-Knows->{as:a} RETURN a"),
]


def _cols(q):
    return [c.strip() for c in q.split("RETURN")[1].split(",")]


MODES = {"merge": ("1", "1"), "merge_force": ("1", "force"), "probe": ("1", "0"), "unfused": ("0", "1")}


def _mode(monkeypatch, mode):
    fuse, merge = MODES[mode]
    monkeypatch.setenv("OMX_FUSE_CHECK", fuse)
    monkeypatch.setenv("OMX_MERGE", merge)


@pytest.mark.parametrize("mode", list(MODES))
@pytest.mark.parametrize("q", CYCLES, ids=[q[0] for q in CYCLES])
def test_cycle_parity(rmat10, q, mode, monkeypatch):
    _mode(monkeypatch, mode)
    g, ref = rmat10
    _parity(g, ref, q[1], _cols(q[1]))


@pytest.mark.parametrize("q", CYCLES, ids=[q[0] for q in CYCLES])
def test_fused_counts_equal_unfused(rmat10, q, monkeypatch):
    import orientdb_amd as o
    g, _ = rmat10
    info = {}
    for mode in MODES:
        _mode(monkeypatch, mode)
        info[mode] = o.OMatchStatement(q[1]).execute(g).info
    for mode in ("merge", "merge_force", "probe"):
        for k in ("n_rows", "bindings", "edges_traversed"):
            assert info[mode][k] == info["unfused"][k], (mode, k)


@pytest.mark.parametrize("q", CYCLES, ids=[q[0] for q in CYCLES])
def test_shorter_list_first_equals_plain_fused(rmat10, q, monkeypatch):
    """The fused check iterates the shorter of N_x(x), N_y(y) (exec.hip expand_check_swapped); with
    that disabled (OMX_SWAP_CHECK=0) every row expands N_x(x): same rows, bindings and E_t."""
    import orientdb_amd as o
    g, ref = rmat10
    info = {}
    for sw in ("1", "0"):
        monkeypatch.setenv("OMX_SWAP_CHECK", sw)
        rs = _parity(g, ref, q[1], _cols(q[1]))
        info[sw] = rs.info
    for k in ("n_rows", "bindings", "edges_traversed"):
        assert info["1"][k] == info["0"][k], k


@pytest.mark.parametrize("merge", ["0", "force"])
@pytest.mark.parametrize("q", CYCLES[:3], ids=[q[0] for q in CYCLES[:3]])
def test_cycle_parity_heavy_and_multigraph(rmat10, rmat10_raw, q, merge, monkeypatch):
    """every probed row of degree ≥ 2 through the chunked kernel's fused path, or every row merged;
    parallel edges kept (a merged row keeps N_x's multiplicity: one row per edge x → t, P/OMatchStatement
    .java:468-477 checks each of them for existence)."""
    import orientdb_amd as o
    monkeypatch.setenv("OMX_HEAVY_DEG", "2")
    monkeypatch.setenv("OMX_MERGE", merge)
    for g, ref in (rmat10, rmat10_raw):
        rs = _parity(g, ref, q[1], _cols(q[1]))
        monkeypatch.setenv("OMX_FUSE_CHECK", "0")
        un = o.OMatchStatement(q[1]).execute(g).info
        monkeypatch.setenv("OMX_FUSE_CHECK", "1")
        for k in ("n_rows", "bindings", "edges_traversed"):
            assert rs.info[k] == un[k], k


@pytest.mark.parametrize("mode", list(MODES))
def test_fused_check_after_set_valued_hop_multigraph(rmat10_raw, mode, monkeypatch):
    """On the multigraph the hop b → c into a node with a WHERE is set-valued (P/OMatchPathItem.java:61,
    71-78: a c reached over parallel edges binds once, Step::distinct_nb), so the closing check c → a
    cannot be fused into it per edge: every mode gives the oracle's rows and bindings."""
    _mode(monkeypatch, mode)
    g, ref = rmat10_raw
    q = CYCLES[1][1]
    _parity(g, ref, q, _cols(q))


_TRI16 = {}


@pytest.mark.parametrize("merge", ["1", "force", "0"])
def test_filtered_triangle_rmat16(rmat16, merge, monkeypatch):
    """A filtered fused triangle at RMAT-16 (longer lists than RMAT-10: hubs of degree ~10^3) with the merge
    chosen by its ratio rule, forced, and off; row count, digest of the rows, E_t and bindings equal
    dfs_ref.c's (the digest instead of a host set of the ~10^6 rows: the same check, without the Python
    set that took most of the test's time)."""
    import orientdb_amd as o
    from oracle import dfs
    monkeypatch.setenv("OMX_MERGE", merge)
    g, ref = rmat16
    q = "MATCH {class:Person,as:a,where:(age < 10)}-Knows->{as:b}-Knows->{as:c,where:(age > 20)}-Knows->{as:a} RETURN a,b,c"
    if "want" not in _TRI16:
        _TRI16["want"] = dfs.run(ref.cg, q, nthreads=8, emit=False, digest=["a", "b", "c"])
    want = _TRI16["want"]
    rs = o.OMatchStatement(q).execute(g, flags=o.OMX_FLAG_KEEP_DEVICE | o.OMX_FLAG_DIGEST, documents=False)
    assert rs.info["n_rows"] > 0
    assert rs.info["digest"] == want["digest"]
    assert rs.info["bindings"] == want["bindings"] and rs.info["edges_traversed"] == want["edges"]


@pytest.mark.parametrize("k", [1, 7, 64, 100, 128, 200])
def test_merge_long_and_short_rows(k, monkeypatch):
    """Merged rows of every size against the probe and a brute-force enumeration: vertex 0 → 1, 1 → s
    and s → 0 for the k vertices s of S, plus chords s → s + 1: the row (0, 1) intersects N_out(1) = S
    ∪ … with N_in(0) = S (m + n = 2k: one row filling a wave tile's half at k = 128, over the merge cap at 200),
    the rows (1, s) and (s, 0) lists of one or two entries (many rows a tile, rows spanning a thread's
    8 merged positions)."""
    import orientdb_amd as o
    V = k + 2
    edges = {(0, 1)} | {(1, s) for s in range(2, V)} | {(s, 0) for s in range(2, V)}
    edges |= {(s, s + 1) for s in range(2, V - 1)}
    out = {v: sorted(t for (u, t) in edges if u == v) for v in range(V)}
    rp = np.zeros(V + 1, np.uint64)
    rp[1:] = np.cumsum([len(out[v]) for v in range(V)])
    col = np.array([t for v in range(V) for t in out[v]], np.uint32)
    g = o.GraphSnapshot.person_knows(rp, col, seed=1, device=0, keep_csr=True)
    q = CYCLES[0][1]
    want = sorted((a, b, c) for (a, b) in edges for c in out[b] if (c, a) in edges)
    res = {}
    for merge in ("force", "1", "0"):
        monkeypatch.setenv("OMX_MERGE", merge)
        rs = o.OMatchStatement(q).execute(g, flags=o.OMX_FLAG_NO_RID_MAP)
        idx = [rs.columns.index(c) for c in "abc"]
        got = sorted(tuple(int(x) for x in row) for row in rs.rows[:, idx].tolist())
        assert got == want, merge
        res[merge] = (rs.info["edges_traversed"], rs.info["bindings"], rs.info["n_rows"])
    assert res["force"] == res["1"] == res["0"]
    g.close()


@pytest.fixture(scope="module")
def ldbc():
    import orientdb_amd as o
    return o.GraphSnapshot.ldbc_like(device=0, keep_csr=True)


@pytest.fixture(scope="module")
def ldbc_ref(ldbc):
    """oracle/dfs_ref.c over the SF10 triangles, computed once for the parametrized device runs (with
    the rows' sorted packed keys)"""
    from oracle import dfs
    g = ldbc
    cg = dfs.CsrGraph(g.csr[0], g.csr[1], {"uid": np.arange(g.V, dtype=np.int64), "age": g.age})
    ref = dfs.run(cg, CYCLES[0][1], nthreads=8)
    ref["key"] = _tri_key(ref["rows"].astype(np.uint64))
    return ref


def _tri_key(m):
    return np.sort((m[:, 0] << np.uint64(42)) | (m[:, 1] << np.uint64(21)) | m[:, 2])


@pytest.mark.parametrize("merge", ["force", "0"])
def test_c4_ldbc_sf10_vs_c_oracle(ldbc, ldbc_ref, merge, monkeypatch):
    """configs[3] at full size: every directed triangle of the LDBC-like SF10 Knows graph, bit-exact
    against oracle/dfs_ref.c, with the same traversed-edge count — merge path on every row that fits a
    tile, and off (the probe, the default; the ratio rule between them is covered at RMAT-10)."""
    import orientdb_amd as o
    monkeypatch.setenv("OMX_MERGE", merge)
    g, ref = ldbc, ldbc_ref
    q = CYCLES[0][1]
    rs = o.OMatchStatement(q).execute(g, flags=o.OMX_FLAG_NO_RID_MAP, documents=False)
    assert rs.info["n_rows"] == len(ref["rows"])
    assert rs.info["edges_traversed"] == ref["edges"]
    idx = [rs.columns.index(c) for c in ref["aliases"]]
    got = rs.rows[:, idx].astype(np.uint64)
    assert np.array_equal(_tri_key(got), ref["key"])
