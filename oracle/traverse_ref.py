"""CPU restatement of the reference's TRAVERSE work list and of SELECT expand() chains.

TEST INFRASTRUCTURE ONLY: `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may
import this module, as the checker; the product path (orientdb_amd, libomx) never does.

What it restates (reference file:line, C/ = core/src/main/java/com/orientechnologies/orient/core/):
  * C/command/traverse/OTraverse.java:83-110 — `next()`: peek the head process of the memory, call its
    `process()`, a non-null return is one result; `hasNext()` stops at `limit` results (:68-70).
  * C/command/traverse/OTraverseContext.java — the memory: a stack (DEPTH_FIRST: push = addFirst) or a
    queue (BREADTH_FIRST: add = addLast); `next()` peeks the first element, `dropFrame()` removes it;
    `pop(record)` also removes the record from the history set (:58-70); `isAlreadyTraversed` /
    `addTraversed` test / add the record (:101-115).
  * C/command/traverse/OTraverseRecordSetProcess.java:40-70 — the FROM records: one record process per
    target record, pushed one per call; the set process pops itself when the target is exhausted.
  * C/command/traverse/OTraverseRecordProcess.java:44-181 — per record: drop it when already in the
    history or when the WHILE predicate is not TRUE; otherwise add it to the history; at MAXDEPTH pop it
    (history entry removed) and return it; else push one process per field value (a multi-value →
    OTraverseMultiValueProcess, a single link → a record process), fields reversed for DEPTH_FIRST,
    and return the record (the frame stays: its next `process()` finds it in the history and drops).
  * C/command/traverse/OTraverseMultiValueProcess.java:38-52 — one record process per element, pushed
    one per call, then pop.
  * C/command/traverse/OTraversePath.java:55-80 — $depth: +1 per record step, fields / indexes keep it,
    the record set is the empty path (depth -1), so a FROM record has depth 0.
  * S/OSQLEngine.java:264-290 (S/ = C/sql/) — foreachRecord: a method call on a multi-value concatenates
    every element's result in order (OMultiCollectionIterator), duplicates kept — the `out().out()`
    chains of SELECT expand().

Parity pin: the document tree and expected orders of C/.../traverse/OTraverseTest.java (testDepthTraverse,
testBreadthTraverse; core/src/test/...) are checked against `traverse()` in tests/test_traverse_oracle.py.
No reference run exists for the vertex-graph form (no JVM in this image), so the graph cases are pinned
by that restatement alone ("TRAVERSE parity pinned by OTraverseTest's orders").
"""
from collections import deque

DEPTH_FIRST = "DEPTH_FIRST"
BREADTH_FIRST = "BREADTH_FIRST"


class _Memory:
    """OTraverseContext.StackMemory / QueueMemory (OTraverseContext.java:150-224)."""

    def __init__(self, strategy):
        self.d = deque()
        self.breadth = strategy == BREADTH_FIRST

    def add(self, p):
        if self.breadth:
            self.d.append(p)      # QueueMemory.add: addLast
        else:
            self.d.appendleft(p)  # StackMemory.add: push (addFirst)

    def next(self):
        return self.d[0] if self.d else None  # peek

    def drop_frame(self):
        if not self.d:
            raise RuntimeError("Traverse stack is empty")
        self.d.popleft()  # removeFirst


class _Traverse:
    def __init__(self, fields_of, predicate, max_depth, strategy, limit):
        self.fields_of = fields_of
        self.predicate = predicate
        self.max_depth = max_depth
        self.strategy = strategy
        self.limit = limit
        self.memory = _Memory(strategy)
        self.history = set()

    # OTraverseContext.pop(record) (:58-70)
    def pop(self, record=None):
        if record is not None:
            self.history.discard(record)
        self.memory.drop_frame()


class _RecordSetProcess:
    def __init__(self, t, records):
        self.t = t
        self.it = iter(records)
        t.memory.add(self)

    def process(self):
        for rec in self.it:
            self.t.memory.add(_RecordProcess(self.t, rec, 0))
            return None
        self.t.pop()
        return None


class _MultiValueProcess:
    def __init__(self, t, values, depth):
        self.t = t
        self.it = iter(values)
        self.depth = depth  # the owning record's path depth (a field keeps it)

    def process(self):
        for v in self.it:
            self.t.memory.add(_RecordProcess(self.t, v, self.depth + 1))
            return None
        self.t.pop()
        return None


class _RecordProcess:
    def __init__(self, t, record, depth):
        self.t = t
        self.record = record
        self.depth = depth

    def process(self):
        t = self.t
        if self.record is None:
            t.pop()
            return None
        if self.record in t.history:  # isAlreadyTraversed → drop()
            t.pop()
            return None
        if t.predicate is not None and t.predicate(self.record, self.depth) is not True:
            t.pop()
            return None
        t.history.add(self.record)
        if t.max_depth > -1 and self.depth == t.max_depth:
            t.pop(self.record)  # pop(): the history entry goes too
        else:
            values = list(t.fields_of(self.record))
            if t.strategy == DEPTH_FIRST:
                values.reverse()
            for v in values:
                if v is None:
                    continue
                if isinstance(v, (list, tuple)):
                    t.memory.add(_MultiValueProcess(t, v, self.depth))
                else:
                    t.memory.add(_RecordProcess(t, v, self.depth + 1))
        return self.record


def traverse(roots, fields_of, predicate=None, max_depth=-1, strategy=DEPTH_FIRST, limit=0):
    """The records OTraverse.execute() returns, in order.

    roots: the FROM records in target order. fields_of(record): the values of the traversed fields in
    field order — None, a record (a link) or a list of records (a multi-value, e.g. out('L')).
    predicate(record, depth) -> bool: the WHILE condition with $depth (None: always).
    """
    t = _Traverse(fields_of, predicate, max_depth, strategy, limit)
    _RecordSetProcess(t, roots)
    out = []
    while True:
        if limit > 0 and len(out) >= limit:
            break
        p = t.memory.next()
        if p is None:
            break
        r = p.process()
        if r is not None:
            out.append(r)
    return out


def csr_lists(rp, col):
    """fields_of helper: v → its CSR row as a list (the ridbag order)."""
    def row(v):
        return [int(x) for x in col[rp[v]:rp[v + 1]]]
    return row


def expand_chain(roots, hops):
    """SELECT expand(h0().h1()...) FROM roots: each hop maps a record to its neighbour list; every hop
    concatenates the lists of the current records in order (OSQLEngine.foreachRecord)."""
    cur = list(roots)
    for h in hops:
        nxt = []
        for r in cur:
            nxt.extend(h(r))
        cur = nxt
    return cur
