"""The TRAVERSE oracle (oracle/traverse_ref.py) against the reference's own golden orders, and the
device's level-synchronous formulation (exec.hip Executor::traverse_bfs) against the oracle's literal
work list on random graphs (CPU only).

The golden orders are OTraverseTest.testDepthTraverse / testBreadthTraverse
(core/src/test/java/com/orientechnologies/orient/core/command/traverse/OTraverseTest.java:45-150):
a root document with links `a`, `b` and a link list `c`, traversed with fields("*").
"""
import random

import pytest

from oracle.traverse_ref import BREADTH_FIRST, DEPTH_FIRST, expand_chain, traverse


def _otraverse_test_docs():
    # document → its fields in insertion order: a link (str) or a link list (list of str)
    return {
        "root": [("a", "a"), ("b", "b"), ("c", ["c1", "c2", "c3"])],
        "a": [("aa", "aa"), ("ab", "ab")],
        "b": [("ba", "ba"), ("bb", "bb")],
        "c1": [("c1a", "c1a"), ("c1b", "c1b")],
        "c2": [("c2a", "c2a"), ("c2b", "c2b")],
        "c3": [("c3a", "c3a"), ("c3b", "c3b")],
    }


def _fields_star(docs):
    return lambda r: [v for _, v in docs.get(r, [])]


def test_golden_depth_first():
    docs = _otraverse_test_docs()
    got = traverse(["root"], _fields_star(docs), strategy=DEPTH_FIRST)
    assert got == ["root", "a", "aa", "ab", "b", "ba", "bb", "c1", "c1a", "c1b", "c2", "c2a", "c2b", "c3", "c3a", "c3b"]


def test_golden_breadth_first():
    docs = _otraverse_test_docs()
    got = traverse(["root"], _fields_star(docs), strategy=BREADTH_FIRST)
    assert got == ["root", "a", "b", "aa", "ab", "ba", "bb", "c1", "c2", "c3", "c1a", "c1b", "c2a", "c2b", "c3a", "c3b"]


def test_maxdepth_repeats_last_level():
    # 0 → [1, 2], 1 → [3], 2 → [3]: at MAXDEPTH the popped record leaves the history, so 3 comes twice
    adj = {0: [1, 2], 1: [3], 2: [3], 3: []}
    f = lambda v: [adj[v]]
    assert traverse([0], f, max_depth=2, strategy=BREADTH_FIRST) == [0, 1, 2, 3, 3]
    assert traverse([0], f, predicate=lambda v, d: d <= 2, strategy=BREADTH_FIRST) == [0, 1, 2, 3]
    assert traverse([0], f, max_depth=0, strategy=BREADTH_FIRST) == [0]
    assert traverse([0, 0], f, max_depth=0, strategy=BREADTH_FIRST) == [0, 0]
    assert traverse([0, 0], f, strategy=BREADTH_FIRST) == [0, 1, 2, 3]


def test_limit_and_predicate_drop():
    adj = {0: [1, 2], 1: [2, 3], 2: [0], 3: [1]}
    f = lambda v: [adj[v]]
    assert traverse([0], f, strategy=BREADTH_FIRST, limit=3) == [0, 1, 2]
    # a record failing WHILE is not remembered: reached again at another depth, it is re-tested
    p = lambda v, d: not (v == 2 and d == 1)
    assert traverse([0], f, predicate=p, strategy=BREADTH_FIRST) == [0, 1, 2, 3]


def level_sync(roots, adj, pred=None, max_depth=-1, limit=0):
    """The device formulation: per level, keep the entries not in the history that pass WHILE($depth);
    below MAXDEPTH only each record's first entry, which joins the history; at MAXDEPTH every entry."""
    hist = set()
    out = []
    cur = list(roots)
    d = 0
    while cur:
        last = max_depth >= 0 and d == max_depth
        acc = []
        claimed = set()
        for w in cur:
            if w in hist or (pred is not None and not pred(w, d)):
                continue
            if not last:
                if w in claimed:
                    continue
                claimed.add(w)
            acc.append(w)
        if not last:
            hist.update(acc)
        out.extend(acc)
        if last or not acc or (limit > 0 and len(out) >= limit):
            break
        cur = [x for w in acc for x in adj[w]]
        d += 1
    return out[:limit] if limit > 0 else out


@pytest.mark.parametrize("seed", range(40))
def test_level_sync_equals_work_list(seed):
    rnd = random.Random(seed)
    V = rnd.randint(1, 40)
    adj = {v: [rnd.randrange(V) for _ in range(rnd.randint(0, 5))] for v in range(V)}
    roots = [rnd.randrange(V) for _ in range(rnd.randint(1, 4))]
    prop = [rnd.randrange(100) for _ in range(V)]
    preds = [None, lambda v, d: d < 3, lambda v, d: prop[v] < 70, lambda v, d: d != 1 or prop[v] < 50,
             lambda v, d: d % 2 == 0 or prop[v] > 30]
    pred = preds[seed % len(preds)]
    max_depth = [-1, 0, 1, 2, 4][(seed // 5) % 5]
    limit = [0, 0, 3, 7][seed % 4]
    want = traverse(roots, lambda v: [adj[v]], predicate=pred, max_depth=max_depth, strategy=BREADTH_FIRST,
                    limit=limit)
    assert level_sync(roots, adj, pred, max_depth, limit) == want


def test_expand_chain_keeps_order_and_repeats():
    adj = {0: [1, 2], 1: [3], 2: [3, 1], 3: []}
    assert expand_chain([0], [lambda v: adj[v]] * 2) == [3, 3, 1]
    assert expand_chain([0, 0], [lambda v: adj[v]]) == [1, 2, 1, 2]


def _bfs_dist(adj, s):
    dist = {s: 0}
    q = [s]
    for v in q:
        for w in adj[v]:
            if w not in dist:
                dist[w] = dist[v] + 1
                q.append(w)
    return dist


@pytest.mark.parametrize("seed", range(30))
def test_shortest_path_oracle_paths_are_paths(seed):
    """oracle/shortest_path_ref.py: the returned list is a walk from the source to the destination along
    the direction's edges whose length is the BFS distance (the bidirectional search meets on a shortest
    path), and empty exactly when the destination is unreachable (no maxDepth)."""
    from oracle.shortest_path_ref import shortest_path
    rnd = random.Random(seed)
    V = rnd.randint(2, 30)
    out = {v: [rnd.randrange(V) for _ in range(rnd.randint(0, 3))] for v in range(V)}
    inn = {v: [] for v in range(V)}
    for v in range(V):
        for w in out[v]:
            inn[w].append(v)
    s, t = rnd.randrange(V), rnd.randrange(V)
    p = shortest_path(s, t, lambda v: out[v], lambda v: inn[v])
    d = _bfs_dist(out, s)
    if t not in d:
        assert p == []
        return
    assert p[0] == s and p[-1] == t
    assert all(b in out[a] for a, b in zip(p, p[1:]))
    assert len(p) - 1 == d[t]
