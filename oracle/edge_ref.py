"""TEST INFRASTRUCTURE — a CPU restatement (numpy) of the edge-node 2-hop

    MATCH {class:Person, as:a, where:(A)}.outE('L'){as:e, where:(W)}.inV(){as:b, where:(B)} RETURN a, e, b

over an out-CSR whose entries are the edge records (entry i = record i, per-record fields as arrays), for
the parity tests and the E1 line's CPU baseline (bench.py). It follows the reference's semantics as
oracle/match_ref.py restates them: outE() from a vertex yields the edge records of its out_<L> ridbag
(OSQLFunctionMove.v2e, GF/OSQLFunctionMove.java:109-121), inV() from an edge record its `in` vertex
(e2v, :122-144), and every forward step keeps the targets passing their alias's WHERE
(OMatchPathItem.executeTraversal, P/OMatchPathItem.java:49-78). Rows are distinct by construction (an
edge record has one source and one target). E_t = Σ deg(a) over the roots (the v2e
step's entries) + one entry per kept edge record (the e2v step). Checked against match_ref.py by
tests/test_oracle_edge_ref.py. Never imported by the product.
"""
import numpy as np


def edge_two_hop(rp, col, roots, emask, bmask, rows=True):
    """roots: vertex ids (int array); emask: bool per edge record (W); bmask: bool per vertex (B).
    Returns (a, e, b) arrays (None when rows=False) and E_t."""
    rp = np.asarray(rp, dtype=np.int64)
    roots = np.asarray(roots, dtype=np.int64)
    lo, hi = rp[roots], rp[roots + 1]
    deg = hi - lo
    n = int(deg.sum())
    if n == 0:
        return (np.zeros(0, np.int64),) * 3 if rows else None, 0
    # every root's entries: lo[r] + 0..deg[r)-1
    starts = np.repeat(lo - np.concatenate(([0], np.cumsum(deg)[:-1])), deg)
    e = starts + np.arange(n, dtype=np.int64)
    src = np.repeat(roots, deg)
    keep = emask[e]
    e, src = e[keep], src[keep]
    b = np.asarray(col, dtype=np.int64)[e]
    edges = n + int(e.size)
    keep = bmask[b]
    if not rows:
        return None, edges
    return (src[keep], e[keep], b[keep]), edges
