"""The set-based CPU baseline (oracle/set_ref.c, bench.py cpu_baseline `set_based`) computes the same
bindings as the DFS restatement oracle/dfs_ref.c (itself pinned to match_ref.py by
tests/test_oracle_dfs_pin.py): equal complete bindings, E_t, result rows and digest, on simple graphs and
multigraphs (a filtered forward hop is set-valued, P/OMatchPathItem.java:61,71-78)."""
import numpy as np
import pytest

CHAINS = [
    ("c2_both_ends", "MATCH {class:Person,as:a,where:(age < 5)}-Knows->{as:b}-Knows->{as:c,where:(age >= 90)} RETURN a,b,c",
     ["a", "b", "c"]),
    ("m1_shape", "MATCH {class:Person,as:a,where:(age < 1)}-Knows->{as:b}-Knows->{as:c,where:(age >= 90)} RETURN a,b,c",
     ["a", "b", "c"]),
    ("c1_abc", "MATCH {class:Person,as:a,where:(age < 20)}-Knows->{as:b}-Knows->{as:c} RETURN a,b,c", ["a", "b", "c"]),
    ("three_hop", "MATCH {class:Person,as:a,where:(uid < 40)}-Knows->{as:b}-Knows->{as:c}-Knows->{as:d,where:(age<10)} RETURN a,b,c,d",
     ["a", "b", "c", "d"]),
    ("in_filtered", "MATCH {class:Person,as:a,where:(age < 8)}.in('Knows'){as:b,where:(age < 60)}.in('Knows'){as:c} RETURN a,b,c",
     ["a", "b", "c"]),
    ("mid_filter", "MATCH {class:Person,as:a,where:(age < 10)}-Knows->{as:b,where:(age > 30)}-Knows->{as:c} RETURN a,b,c",
     ["a", "b", "c"]),
]


@pytest.fixture(scope="module", params=[True, False], ids=["simple", "multigraph"])
def g11(request):
    import orientdb_amd as o
    from oracle import dfs
    rp, col = o.rmat_csr(11, 16, 11, request.param)
    age = o.synthetic_int_column(1 << 11, 11 ^ 0xA9E, 100).astype(np.int64)
    return dfs.CsrGraph(rp, col, {"uid": np.arange(1 << 11, dtype=np.int64), "age": age}, simple=request.param)


@pytest.mark.parametrize("q", CHAINS, ids=[q[0] for q in CHAINS])
def test_set_based_equals_dfs(g11, q):
    from oracle import dfs
    _, query, cols = q
    want = dfs.run(g11, query, nthreads=4, digest=cols)
    got = dfs.set_run(g11, query, nthreads=4, digest=cols, rows=True)
    assert got["bindings"] == want["bindings"]
    assert got["edges"] == want["edges"]
    assert got["digest"] == want["digest"]  # every binding hashed, in both
    rows = np.unique(got["rows"], axis=0)
    assert np.array_equal(rows, want["rows"])


def test_set_based_distinct_column(g11):
    """configs[0]'s shape: RETURN fof marks the last hop's union of lists in a V-bit set."""
    from oracle import dfs
    q = "MATCH {class:Person}-Knows->{}-Knows->{as:fof} RETURN fof"
    want = dfs.run(g11, q, nthreads=4, emit=False, distinct="fof")
    got = dfs.set_run(g11, q, nthreads=4, distinct="fof")
    assert got["bindings"] == want["bindings"] and got["edges"] == want["edges"]
    assert np.array_equal(got["distinct"], want["distinct"])


def test_set_based_root_sample_and_threads(g11):
    from oracle import dfs
    q = CHAINS[0][1]
    a = dfs.set_run(g11, q, nthreads=1, root_sample=7, digest=["a", "b", "c"])
    b = dfs.set_run(g11, q, nthreads=8, root_sample=7, digest=["a", "b", "c"])
    w = dfs.run(g11, q, nthreads=2, root_sample=7, emit=False, digest=["a", "b", "c"])
    assert a["nroots"] == 7 and a["bindings"] == b["bindings"] == w["bindings"]
    assert a["digest"] == b["digest"] == w["digest"]


def test_set_based_refuses_closing_checks(g11):
    from oracle import dfs
    with pytest.raises(NotImplementedError):
        dfs.set_run(g11, "MATCH {class:Person,as:a}-Knows->{as:b}-Knows->{as:c}-Knows->{as:a} RETURN a,b,c")
