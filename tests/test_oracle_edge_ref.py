"""oracle/edge_ref.py (the E1 CPU baseline's restatement) against oracle/match_ref.py on RMAT graphs whose
Knows edges are records with a field `w` (rows as RID tuples, E_t as the oracle counts it)."""
import numpy as np
import pytest

from oracle.edge_ref import edge_two_hop
from oracle.match_ref import MatchOracle
from tests.rmat_oracle import refdb_from_csr


@pytest.mark.parametrize("scale,amax,wmax,bmin", [(7, 20, 30, 50), (8, 5, 60, 80)])
def test_edge_ref_matches_match_ref(scale, amax, wmax, bmin):
    import orientdb_amd as o
    from orientdb_amd.graph import rmat_csr
    rp, col = rmat_csr(scale, seed=scale)
    V, E = len(rp) - 1, len(col)
    age = o.synthetic_int_column(V, 17, 100)
    w = o.synthetic_int_column(E, 23, 100)
    db = refdb_from_csr(rp, col, age, w)
    q = ("MATCH {class:Person,as:a,where:(age < %d)}.outE('Knows'){as:e, where:(w < %d)}.inV(){as:b, where:(age >= %d)}"
         " RETURN a, e, b" % (amax, wmax, bmin))
    orc = MatchOracle(db, q)
    want = {((11 << 48) | r[0].rid[1], (12 << 48) | r[1].rid[1], (11 << 48) | r[2].rid[1])
            for r in ([row["a"], row["e"], row["b"]] for row in orc.execute())}
    (a, e, b), edges = edge_two_hop(rp, col, np.nonzero(age < amax)[0], w < wmax, age >= bmin)
    got = {((11 << 48) | int(x), (12 << 48) | int(y), (11 << 48) | int(z)) for x, y, z in zip(a, e, b)}
    assert want and got == want and len(got) == len(a)
    assert edges == orc.stats["edges"]
