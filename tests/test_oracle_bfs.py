"""The C BFS restatement of variable-length items (oracle/bfs_ref.c) agrees with the walk-enumerating
Python oracle (oracle/match_ref.py, the reference's recursion restated) where both run, so it can check
the device path at scales the walk oracle cannot reach (configs[2]: RMAT-24)."""
import numpy as np
import pytest


@pytest.fixture(scope="module")
def rmat9():
    import orientdb_amd as o
    from tests.rmat_oracle import refdb_from_csr
    rp, col = o.rmat_csr(9, 16, 9)
    age = o.synthetic_int_column(512, 9 ^ 0xA9E, 100).astype(np.int64)
    return rp, col, age, refdb_from_csr(rp, col, age)


@pytest.mark.parametrize("depth,where", [(0, None), (1, None), (2, None), (3, "age < 40"), (2, "age >= 50")])
def test_bfs_ball_equals_walk_oracle(rmat9, depth, where):
    from oracle import dfs
    from oracle.match_ref import MatchOracle
    rp, col, age, db = rmat9
    roots = np.array([3, 10, 17, 40, 41, 200], np.uint32)
    wtxt = (", where:(%s)" % where) if where else ""
    q = ("MATCH {class:Person,as:s,where:(uid = ?)}-Knows->{as:v, while:($depth < %d)%s} RETURN s, v" % (depth, wtxt))
    mask = None
    if where:
        k, op, val = where.split()
        mask = {"<": np.less, ">=": np.greater_equal}[op](age, int(val))
    r = dfs.bfs_varlen(rp, col, roots, max_depth=depth, where_mask=mask, nthreads=4)
    got = {(int(roots[i]), int(v)) for i, v in r["pairs"]}
    want = set()
    for root in roots:
        for row in MatchOracle(db, q).execute([int(root)]):
            want.add((row["s"].rid[1], row["v"].rid[1]))
    assert got == want and r["n"] == len(want)
