"""Host mirror of the reference's MATCH command interface, executed on the MI355X.

Reference interface (OrientDB 2.2.8):
  db.command(new OCommandSQL("MATCH ...")).execute(args...)            → List<ODocument>
      ODatabaseDocumentTx.command  core/.../db/document/ODatabaseDocumentTx.java:702-714
  OMatchStatement.parse / execute / setLimit
      core/.../sql/parser/OMatchStatement.java:129-178, :231-267, :968-971
  OResultSet (OConcurrentResultSet)  core/.../sql/query/OResultSet.java:33

Here: GraphDatabase(snapshot).command(OCommandSQL("MATCH ...")).execute(*args) → OResultSet of
ODocument (alias → ORecordId), or of ORecordId for $elements/$pathElements. Errors keep the
reference's split: OmxParseError ≈ OCommandSQLParsingException, OmxExecutionError ≈
OCommandExecutionException, OmxUnsupported = "not executable by the device engine" (the Java
strategy falls back to OMatchStatement).
"""
import ctypes as C
import json
import re

import numpy as np

from . import _native as N
from .graph import unpack_rid

_RID_RE = re.compile(r"^#(-?\d+):(\d+)$")


class ORecordId(tuple):
    """#cluster:position (C/id/ORecordId.java)."""

    def __new__(cls, cluster, position):
        return super().__new__(cls, (int(cluster), int(position)))

    @classmethod
    def from_packed(cls, r):
        """None for a null binding (an unmatched optional node, OMX_NULL_RID)."""
        if int(r) == N.OMX_NULL_RID:
            return None
        return cls(*unpack_rid(r))

    @classmethod
    def parse(cls, s):
        """'#cluster:position' → ORecordId, or None if s is not a RID string."""
        m = _RID_RE.match(s)
        return cls(int(m.group(1)), int(m.group(2))) if m else None

    @property
    def cluster(self):
        return self[0]

    @property
    def position(self):
        return self[1]

    def packed(self):
        return (self[0] << 48) | self[1]

    def __repr__(self):
        return "#%d:%d" % self


class ODocument(dict):
    def field(self, name):
        return self.get(name)

    def fieldNames(self):
        return list(self.keys())


class OResultSet(list):
    """Distinct result rows + execution statistics (edges traversed, bindings, timings)."""
    info = None
    kernel_stats = None
    kernel_launches = None
    columns = None
    rows = None  # numpy u64 [n, k] of packed RIDs
    cells = None  # document results: {column: (OMX_CELL_* int32 [n], value bits u64 [n])}


def _values(args, named):
    vals = []
    for i, a in enumerate(args):
        vals.append(_value(a, index=i))
    for k, a in (named or {}).items():
        vals.append(_value(a, name=k))
    arr = (N.omx_value * max(1, len(vals)))(*vals)
    return arr, len(vals)


def _value(a, index=0, name=None):
    v = N.omx_value()
    v.index = index
    v.name = name.encode() if name else None
    if a is None:
        v.type = N.OMX_VAL_NULL
    elif isinstance(a, bool):
        v.type, v.i = N.OMX_VAL_BOOL, int(a)
    elif isinstance(a, (int, np.integer)):
        v.type, v.i = N.OMX_VAL_INT, int(a)
    elif isinstance(a, (float, np.floating)):
        v.type, v.d = N.OMX_VAL_DOUBLE, float(a)
    else:
        v.type, v.s = N.OMX_VAL_STRING, str(a).encode()
    return v


def _json_value(x):
    """A LIST / MAP cell (JSON text): record links come as '#cluster:position' strings."""
    if isinstance(x, str):
        r = ORecordId.parse(x)
        return r if r is not None else x
    if isinstance(x, list):
        return [_json_value(y) for y in x]
    if isinstance(x, dict):
        return ODocument((k, _json_value(v)) for k, v in x.items())
    return x


def _cell_value(cell):
    t = cell.type
    if t == N.OMX_CELL_NULL:
        return None
    if t == N.OMX_CELL_INT:
        return int(cell.i)
    if t == N.OMX_CELL_DOUBLE:
        return float(cell.d)
    if t == N.OMX_CELL_STRING:
        return cell.s.decode("utf-8")
    if t == N.OMX_CELL_BOOL:
        return bool(cell.i)
    if t == N.OMX_CELL_RID:
        return ORecordId.from_packed(cell.rid)
    return _json_value(json.loads(cell.s.decode("utf-8")))


def _column_values(r, c, types, bits):
    """One result column (omx_result_column's types / bits) as ODocument field values; strings, lists
    and maps come through omx_result_cell."""
    out = [None] * len(types)
    ints, dbls = bits.view(np.int64), bits.view(np.float64)
    for t in np.unique(types).tolist():
        idx = np.flatnonzero(types == t)
        if t == N.OMX_CELL_NULL:
            continue
        if t == N.OMX_CELL_INT:
            vs = ints[idx].tolist()
        elif t == N.OMX_CELL_DOUBLE:
            vs = dbls[idx].tolist()
        elif t == N.OMX_CELL_BOOL:
            vs = [bool(x) for x in ints[idx].tolist()]
        elif t == N.OMX_CELL_RID:
            vs = [ORecordId.from_packed(x) for x in bits[idx].tolist()]
        else:
            cell, vs = N.omx_cell(), []
            for i in idx.tolist():
                N.check(N.lib().omx_result_cell(r, i, c, C.byref(cell)))
                vs.append(_cell_value(cell))
        for i, v in zip(idx.tolist(), vs):
            out[i] = v
    return out


class OMatchStatement:
    """OMatchStatement (P/OMatchStatement.java:29) as a drop-in execution strategy."""

    KEYWORD_MATCH = "MATCH"

    def __init__(self, text=None):
        self._h = None
        self._limit = -1
        self.text = None
        if text is not None:
            self.parse(text)

    def parse(self, request):
        text = request.text if isinstance(request, OCommandSQL) else str(request)
        h = C.c_void_p()
        N.check(N.lib().omx_statement_parse(text.encode(), C.byref(h)))
        self.free()
        self._h = h
        self.text = text
        return self

    def setLimit(self, n):
        """limitFromProtocol (:968-971)."""
        self._limit = int(n)
        return self

    def explain(self, graph, *args, **named):
        arr, n = _values(args, named)
        buf = C.create_string_buffer(1 << 16)
        N.check(N.lib().omx_statement_explain(self._h, graph.handle, arr, n, buf, len(buf)))
        return json.loads(buf.value.decode())

    def execute(self, graph, *args, mode=N.OMX_MODE_MATERIALIZE, flags=0, shard=(0, 1), documents=True, comm=None,
                fetch_rows=True, **named):
        """comm: the ranks' Comm (orientdb_amd.dist) when `graph` is a partition; every rank then
        returns its share of the distinct rows (their union is the result). fetch_rows=False leaves the
        RID rows libomx copied to the host unread (rs.rows stays empty; info and timings are read)."""
        arr, n = _values(args, named)
        o = N.omx_exec_options()
        N.lib().omx_exec_options_init(C.byref(o))
        o.mode = mode
        o.flags = flags
        o.limit = self._limit
        o.shard_rank, o.shard_world = shard
        o.params = arr
        o.n_params = n
        o.comm = comm.handle if comm is not None else None
        r = C.c_void_p()
        N.check(N.lib().omx_execute(graph.handle, self._h, C.byref(o), C.byref(r)))
        try:
            return self._collect(r, documents, fetch_rows)
        finally:
            N.lib().omx_result_free(r)

    @staticmethod
    def _collect(r, documents, fetch_rows=True):
        L = N.lib()
        info = N.omx_result_info()
        N.check(L.omx_result_info_get(r, C.byref(info)))
        rs = OResultSet()
        rs.info = {f: getattr(info, f) for f, _ in N.omx_result_info._fields_}
        cols = []
        i = 0
        while True:
            nm = L.omx_result_column_name(r, i)
            if nm is None:
                break
            cols.append(nm.decode())
            i += 1
        rs.columns = cols
        stats = []
        i = 0
        while True:
            name, launches, ms, by = C.c_char_p(), C.c_int64(), C.c_double(), C.c_uint64()
            if L.omx_result_kernel_stat(r, i, C.byref(name), C.byref(launches), C.byref(ms), C.byref(by)) != 0:
                break
            stats.append({"name": name.value.decode(), "launches": launches.value, "ms": ms.value, "alg_bytes": by.value})
            i += 1
        rs.kernel_stats = stats
        launches = []
        i = 0
        while True:
            name, ms, by = C.c_char_p(), C.c_double(), C.c_uint64()
            if L.omx_result_kernel_launch(r, i, C.byref(name), C.byref(ms), C.byref(by)) != 0:
                break
            hbm = C.c_uint64()
            L.omx_result_kernel_launch_bytes(r, i, None, C.byref(hbm))
            launches.append({"name": name.value.decode(), "ms": ms.value, "alg_bytes": by.value, "hbm_bytes": hbm.value})
            i += 1
        rs.kernel_launches = launches
        nrows, ncols = info.n_rows, info.n_cols
        if info.documents:  # RETURN expressions / JSON: one document per row, read column by column
            rs.rows = np.zeros((0, 0), np.uint64)
            rs.cells = {}
            for c, name in enumerate(cols):
                types, bits = np.empty(nrows, np.int32), np.empty(nrows, np.uint64)
                N.check(L.omx_result_column(r, c, types.ctypes.data_as(C.c_void_p), bits.ctypes.data_as(C.c_void_p)))
                rs.cells[name] = (types, bits)
            if documents and nrows:
                vals = [_column_values(r, c, *rs.cells[name]) for c, name in enumerate(cols)]
                rs.extend(ODocument(zip(cols, row)) for row in zip(*vals))
            return rs
        p = L.omx_result_rows(r) if fetch_rows else None
        if p and nrows and ncols:
            rs.rows = np.ctypeslib.as_array(p, shape=(nrows * ncols,)).reshape(nrows, ncols).copy()
        else:
            rs.rows = np.zeros((0, max(ncols, 0)), np.uint64)
        if documents and rs.rows.shape[0]:
            if cols and cols[0] in ("$elements", "$pathElements", "@rid"):  # records (also TRAVERSE / SELECT expand)
                rs.extend(ORecordId.from_packed(x) for x in rs.rows[:, 0])
            else:
                for row in rs.rows:
                    rs.append(ODocument((c, ORecordId.from_packed(x)) for c, x in zip(cols, row)))
        return rs

    def free(self):
        if self._h is not None:
            N.lib().omx_statement_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class OCommandExecutorSQLTraverse(OMatchStatement):
    """`TRAVERSE <out|in|both>('L') FROM <rid|[rids]|class> [WHILE <cond>] [MAXDEPTH d] [LIMIT n]
    STRATEGY BREADTH_FIRST` (S/OCommandExecutorSQLTraverse.java:64-139, C/command/traverse/OTraverse.java):
    the records in the reference's emission order, as ORecordId. DEPTH_FIRST, `*`, several fields and
    sub-query targets raise OmxUnsupported (the host keeps the reference executor for those)."""

    KEYWORD_TRAVERSE = "TRAVERSE"


class OCommandExecutorSQLSelectExpand(OMatchStatement):
    """`SELECT expand(<out|in|both>('L')[.<out|in|both>('L')]*) FROM <target> [WHERE <cond>] [LIMIT n]`:
    every call moves the whole list, duplicates and order kept (S/OSQLEngine.java:264-290)."""

    KEYWORD_SELECT = "SELECT"


class OCommandSQL:
    """OCommandSQL: the text of a command (core/.../sql/OCommandSQL.java)."""

    def __init__(self, text):
        self.text = text


class _BoundCommand:
    def __init__(self, db, request):
        self.db = db
        self.request = request
        self._limit = -1

    def setLimit(self, n):
        self._limit = n
        return self

    def execute(self, *args, **named):
        text = self.request.text.strip()
        word = text.split(None, 1)[0].upper() if text else ""
        if word not in (OMatchStatement.KEYWORD_MATCH, OCommandExecutorSQLTraverse.KEYWORD_TRAVERSE,
                        OCommandExecutorSQLSelectExpand.KEYWORD_SELECT):
            raise N.OmxUnsupported(N.OMX_E_UNSUPPORTED, "only MATCH, TRAVERSE and SELECT expand() run on the device engine")
        st = OMatchStatement(text).setLimit(self._limit)
        try:
            return st.execute(self.db.snapshot, *args, **named)
        finally:
            st.free()


class GraphDatabase:
    """`db.command(new OCommandSQL(...)).execute(...)` over a GraphSnapshot."""

    def __init__(self, snapshot):
        self.snapshot = snapshot

    def command(self, request):
        if isinstance(request, str):
            request = OCommandSQL(request)
        return _BoundCommand(self, request)
