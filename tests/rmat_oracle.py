"""Oracle-side database for synthetic RMAT graphs: the same Person/Knows schema and properties as
GraphSnapshot.rmat, as oracle RefDB records (test infrastructure)."""
import numpy as np

from oracle.match_ref import RefDB


def refdb_from_csr(rp, col, age, w=None):
    db = RefDB()
    # clusters as GraphSnapshot.rmat: V 9, E 10, Person 11 (RID #11:v), Knows 12
    db.create_class("V", cluster=9)
    db.create_class("E", is_edge=True, cluster=10)
    db.create_class("Person", "V", cluster=11)
    db.create_class("Knows", "E", is_edge=True, cluster=12)
    V = len(rp) - 1
    for v in range(V):
        db.add_vertex("Person", {"uid": v, "age": int(age[v])})
    rp = np.asarray(rp, dtype=np.int64)
    for u in range(V):
        for e in range(rp[u], rp[u + 1]):
            db.add_edge("Knows", db.vertices[u], db.vertices[int(col[e])], None if w is None else {"w": int(w[e])})
    return db
