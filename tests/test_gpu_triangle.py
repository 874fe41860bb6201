"""Cyclic patterns (configs[3]): the expansion that binds the last alias of a cycle and the
check that closes it run fused — every expanded neighbour is kept only if it lies in the sorted adjacency
of the row's closing vertex (binary search inside the expansion kernels), so wedges are never
materialised. Parity: identical rows to the oracle and to the unfused expand + check path, and the same
traversed-edge count (the fused kernels add Σ |N(closing vertex)| over the wedges, as the check would).
"""
import numpy as np
import pytest

from tests.test_gpu_parity import _parity, gpu_set, rmat10, rmat10_raw  # noqa: F401  (fixtures)

pytestmark = pytest.mark.gpu

CYCLES = [
    ("triangle", "MATCH {class:Person,as:a}-Knows->{as:b}-Knows->{as:c}-Knows->{as:a} RETURN a,b,c"),
    ("triangle_where_c", "MATCH {class:Person,as:a,where:(age < 30)}-Knows->{as:b}-Knows->{as:c,where:(age > 20)}-Knows->{as:a} RETURN a,b,c"),
    ("triangle_where_b", "MATCH {class:Person,as:a}-Knows->{as:b,where:(age < 50)}-Knows->{as:c}-Knows->{as:a} RETURN a,b,c"),
    ("triangle_in", "MATCH {class:Person,as:a,where:(uid < 300)}<-Knows-{as:b}<-Knows-{as:c}<-Knows-{as:a} RETURN a,b,c"),
    ("triangle_both", "MATCH {class:Person,as:a,where:(uid < 40)}-Knows-{as:b}-Knows-{as:c}-Knows-{as:a} RETURN a,b,c"),
    ("square", "MATCH {class:Person,as:a,where:(uid < 100)}-Knows->{as:b}-Knows->{as:c}-Knows->{as:d}-Knows->{as:a} RETURN a,b,c,d"),
    ("triangle_project", "MATCH {class:Person,as:a}-Knows->{as:b}-Knows->{as:c}-Knows->{as:a} RETURN a"),
]


def _cols(q):
    return [c.strip() for c in q.split("RETURN")[1].split(",")]


@pytest.mark.parametrize("fuse", ["1", "0"])
@pytest.mark.parametrize("q", CYCLES, ids=[q[0] for q in CYCLES])
def test_cycle_parity(rmat10, q, fuse, monkeypatch):
    monkeypatch.setenv("OMX_FUSE_CHECK", fuse)
    g, ref = rmat10
    _parity(g, ref, q[1], _cols(q[1]))


@pytest.mark.parametrize("q", CYCLES, ids=[q[0] for q in CYCLES])
def test_fused_counts_equal_unfused(rmat10, q, monkeypatch):
    import orientdb_amd as o
    g, _ = rmat10
    info = {}
    for fuse in ("1", "0"):
        monkeypatch.setenv("OMX_FUSE_CHECK", fuse)
        info[fuse] = o.OMatchStatement(q[1]).execute(g).info
    for k in ("n_rows", "bindings", "edges_traversed"):
        assert info["1"][k] == info["0"][k], k


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


@pytest.mark.parametrize("q", CYCLES[:3], ids=[q[0] for q in CYCLES[:3]])
def test_cycle_parity_heavy_and_multigraph(rmat10, rmat10_raw, q, monkeypatch):
    """every row of degree ≥ 2 through the chunked kernel's fused path; parallel edges kept."""
    monkeypatch.setenv("OMX_HEAVY_DEG", "2")
    for g, ref in (rmat10, rmat10_raw):
        _parity(g, ref, q[1], _cols(q[1]))


@pytest.fixture(scope="module")
def ldbc():
    import orientdb_amd as o
    return o.GraphSnapshot.ldbc_like(device=0, keep_csr=True)


def test_c4_ldbc_sf10_vs_c_oracle(ldbc):
    """configs[3] at full size: every directed triangle of the LDBC-like SF10 Knows graph, bit-exact
    against oracle/dfs_ref.c, with the same traversed-edge count."""
    import orientdb_amd as o
    from oracle import dfs
    g = ldbc
    q = CYCLES[0][1]
    rs = o.OMatchStatement(q).execute(g, flags=o.OMX_FLAG_NO_RID_MAP)
    cg = dfs.CsrGraph(g.csr[0], g.csr[1], {"uid": np.arange(g.V, dtype=np.int64), "age": g.age})
    ref = dfs.run(cg, q, nthreads=8)
    assert rs.info["n_rows"] == len(ref["rows"])
    assert rs.info["edges_traversed"] == ref["edges"]
    idx = [rs.columns.index(c) for c in ref["aliases"]]
    got = rs.rows[:, idx].astype(np.uint64)
    key = lambda m: np.sort((m[:, 0] << np.uint64(42)) | (m[:, 1] << np.uint64(21)) | m[:, 2])
    assert np.array_equal(key(got), key(ref["rows"].astype(np.uint64)))
