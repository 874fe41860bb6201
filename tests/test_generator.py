"""The synthetic inputs are a pure function of (scale, seed): a numpy restatement of
the generator in orientdb_amd/csrc/gen.cpp reproduces libomx's RMAT edges and property column."""
import numpy as np

M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(x):
    with np.errstate(over="ignore"):
        x = (x + np.uint64(0x9E3779B97F4A7C15))
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return x ^ (x >> np.uint64(31))


def rmat_edges(scale, edge_factor, seed):
    V = 1 << scale
    M = edge_factor * V
    sd = np.uint64(seed)
    mask = np.uint64((1 << scale) - 1)
    m1 = splitmix64(np.uint64(seed ^ 0x1111)) | np.uint64(1)
    m2 = splitmix64(np.uint64(seed ^ 0x2222)) | np.uint64(1)
    c1 = splitmix64(np.uint64(seed ^ 0x3333))
    c2 = splitmix64(np.uint64(seed ^ 0x4444))
    TA, TB, TC = int(0.57 * 4294967296.0), int(0.76 * 4294967296.0), int(0.95 * 4294967296.0)
    i = np.arange(M, dtype=np.uint64)
    with np.errstate(over="ignore"):
        st = sd * np.uint64(0x9E3779B97F4A7C15) + i * np.uint64(0xD1B54A32D192ED03)
        a = np.zeros(M, np.uint64)
        b = np.zeros(M, np.uint64)
        r = None
        for lvl in range(scale):
            if lvl % 2 == 0:
                r = splitmix64(st + np.uint64(lvl))
            x = (r >> np.uint64(32)) if lvl % 2 else (r & np.uint64(0xFFFFFFFF))
            q = np.where(x < TA, 0, np.where(x < TB, 1, np.where(x < TC, 2, 3))).astype(np.uint64)
            a = (a << np.uint64(1)) | (q >> np.uint64(1))
            b = (b << np.uint64(1)) | (q & np.uint64(1))
        h = np.uint64(scale // 2 + 1)

        def scramble(x):
            x = (x * m1 + c1) & mask
            x ^= x >> h
            x = (x * m2 + c2) & mask
            x ^= x >> h
            return x & mask

    return scramble(a).astype(np.int64), scramble(b).astype(np.int64)


def test_rmat_raw_edges_match_restatement():
    import orientdb_amd as o
    u, v = rmat_edges(8, 16, 8)
    rp, col = o.rmat_csr(8, 16, 8, simple=False)
    src = np.repeat(np.arange(256), np.diff(rp.astype(np.int64)))
    got = np.lexsort((col, src))
    want = np.lexsort((v, u))
    assert np.array_equal(src[got], u[want]) and np.array_equal(col[got].astype(np.int64), v[want])


def test_rmat_simple_is_dedup_without_self_loops():
    import orientdb_amd as o
    u, v = rmat_edges(9, 16, 3)
    keep = u != v
    pairs = np.unique(np.stack([u[keep], v[keep]], 1), axis=0)
    rp, col = o.rmat_csr(9, 16, 3, simple=True)
    src = np.repeat(np.arange(512), np.diff(rp.astype(np.int64)))
    assert np.array_equal(np.stack([src, col.astype(np.int64)], 1), pairs)
    # rows sorted strictly ascending (duplicate-free adjacency → rows distinct by construction)
    for r in range(512):
        row = col[rp[r]:rp[r + 1]]
        assert np.all(np.diff(row.astype(np.int64)) > 0)


def test_scramble_is_a_bijection():
    import orientdb_amd as o
    rp, col = o.rmat_csr(10, 16, 10, simple=False)
    # every vertex id is in range; the id map spreads RMAT's low-id hubs (degree of vertex 0 is not max)
    assert col.max() < 1024
    deg = np.diff(rp.astype(np.int64))
    assert deg.argmax() != 0


def test_synthetic_column():
    import orientdb_amd as o
    V, seed = 1000, 1234
    got = o.synthetic_int_column(V, seed, 100)
    with np.errstate(over="ignore"):
        want = splitmix64(np.uint64(seed) ^ (np.arange(V, dtype=np.uint64) * np.uint64(0xA24BAED4963EE407))) % np.uint64(100)
    assert np.array_equal(got, want.astype(np.int32))


def test_csr_transpose_roundtrip():
    import orientdb_amd as o
    rp, col = o.rmat_csr(9, 8, 1)
    trp, tcol = o.csr_transpose(512, rp, col)
    rrp, rcol = o.csr_transpose(512, trp, tcol)
    assert np.array_equal(rrp, rp) and np.array_equal(rcol, col)
