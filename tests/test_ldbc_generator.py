"""configs[3] input: the LDBC-SNB-like Knows generator (gen.cpp omx_ldbc_knows_generate)."""
import numpy as np


def test_ldbc_like_invariants():
    import orientdb_amd as o
    rp, col = o.ldbc_csr(5000, 120_000, 3)
    V = len(rp) - 1
    assert V == 5000 and abs(len(col) - 120_000) < 0.1 * 120_000
    src = np.repeat(np.arange(V), np.diff(rp.astype(np.int64)))
    assert np.all(src != col)                                     # no self loops
    for v in range(0, V, 97):                                     # rows strictly ascending
        assert np.all(np.diff(col[rp[v]:rp[v + 1]].astype(np.int64)) > 0)
    a, b = np.minimum(src, col), np.maximum(src, col)
    assert len(np.unique(a.astype(np.int64) << 32 | b)) == len(col)  # one directed edge per person pair
    tot = np.bincount(src, minlength=V) + np.bincount(col, minlength=V)
    assert tot.max() > 8 * tot.mean()                             # skewed degrees


def test_ldbc_like_is_deterministic_and_clustered():
    import orientdb_amd as o
    from oracle import dfs
    r1, c1 = o.ldbc_csr(3000, 60_000, 5)
    r2, c2 = o.ldbc_csr(3000, 60_000, 5)
    assert np.array_equal(r1, r2) and np.array_equal(c1, c2)
    cg = dfs.CsrGraph(r1, c1, {"uid": np.arange(3000, dtype=np.int64), "age": np.zeros(3000, np.int64)})
    tri = dfs.run(cg, "MATCH {class:Person,as:a}-Knows->{as:b}-Knows->{as:c}-Knows->{as:a} RETURN a,b,c",
                  nthreads=4, emit=False)["bindings"]
    # far more directed triangles than a degree-preserving random graph would have (a few hundred)
    assert tri > 20_000
