"""Oracle-side database for synthetic RMAT graphs: the same Person/Knows schema and properties as
GraphSnapshot.rmat, as oracle RefDB records (test infrastructure)."""
import numpy as np

from oracle.match_ref import RefDB


def refdb_from_csr(rp, col, age):
    db = RefDB()
    db.create_class("V")
    db.create_class("E", is_edge=True)
    db.create_class("Person", "V")  # cluster 11, as GraphSnapshot.rmat
    db.create_class("Knows", "E", is_edge=True)
    V = len(rp) - 1
    for v in range(V):
        db.add_vertex("Person", {"uid": v, "age": int(age[v])})
    rp = np.asarray(rp, dtype=np.int64)
    for u in range(V):
        for e in range(rp[u], rp[u + 1]):
            db.add_edge("Knows", db.vertices[u], db.vertices[int(col[e])])
    return db
