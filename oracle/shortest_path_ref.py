"""CPU restatement of the reference's shortestPath() SQL function.

TEST INFRASTRUCTURE ONLY: `tests/` may import this module as the checker; the product path (orientdb_amd,
libomx) never does.

Restates GF/OSQLFunctionShortestPath.java (GF/ = graphdb/src/main/java/com/orientechnologies/orient/
graph/sql/functions/):
  * execute :85-200 — source == destination → [source]; the right side walks the opposite direction
    (OUT ↔ IN, BOTH stays); both queues start with their end vertex marked visited; each round walks the
    side whose queue is not longer first, `depth` counts walks, `maxDepth <= depth` stops (checked before
    a round and after its first walk), an empty queue stops;
  * walkLeft / walkRight :232-292 — the queue is drained in order; for each entry its neighbours in
    adjacency order: a neighbour visited by the OTHER side ends the search (its previous / next is set to
    the entry first), a neighbour not visited by this side gets the entry as previous / next, is queued
    for the next level and marked visited;
  * computePath :294-313 — previouses from the meeting vertex back to the source, then nexts on to the
    destination.

No reference run exists in this image (no JVM): parity for shortestPath() is pinned by this restatement
alone ("parity unpinned" against reference outputs).
"""
from collections import deque


def shortest_path(src, dst, left_neighbours, right_neighbours, max_depth=None):
    """left_neighbours(v): v's neighbours in the source side's direction, in adjacency order;
    right_neighbours(v): in the opposite direction (the destination side's walk)."""
    if src == dst:
        return [dst]
    ql, qr = deque([src]), deque([dst])
    lv, rv = {src}, {dst}
    prev, nxt = {}, {}

    def compute_path(n):
        res = deque()
        cur = n
        while cur is not None:
            res.appendleft(cur)
            cur = prev.get(cur)
        cur = n
        while cur is not None:
            cur = nxt.get(cur)
            if cur is not None:
                res.append(cur)
        return list(res)

    def walk_left():
        nonlocal ql
        nq = deque()
        while ql:
            cur = ql.popleft()
            for n in left_neighbours(cur):
                if n in rv:
                    prev[n] = cur
                    return compute_path(n)
                if n not in lv:
                    prev[n] = cur
                    nq.append(n)
                    lv.add(n)
        ql = nq
        return None

    def walk_right():
        nonlocal qr
        nq = deque()
        while qr:
            cur = qr.popleft()
            for n in right_neighbours(cur):
                if n in lv:
                    nxt[n] = cur
                    return compute_path(n)
                if n not in rv:
                    nxt[n] = cur
                    nq.append(n)
                    rv.add(n)
        qr = nq
        return None

    depth = 1
    while True:
        if max_depth is not None and max_depth <= depth:
            break
        if not ql or not qr:
            break
        if len(ql) <= len(qr):
            p = walk_left()
            if p is not None:
                return p
            depth += 1
            if max_depth is not None and max_depth <= depth:
                break
            if not ql:
                break
            p = walk_right()
            if p is not None:
                return p
        else:
            p = walk_right()
            if p is not None:
                return p
            depth += 1
            if max_depth is not None and max_depth <= depth:
                break
            if not qr:
                break
            p = walk_left()
            if p is not None:
                return p
        depth += 1
    return []
