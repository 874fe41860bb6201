"""ORACLE (test infrastructure only) — drives oracle/dfs_ref.c over a Person/Knows CSR graph.

The plan (estimates, sortEdges, bound/candidate/free per edge) comes from the Python restatement
(oracle/match_ref.py, MatchOracle); WHERE clauses are evaluated with numpy over the property columns
(same operator semantics as match_ref.Evaluator for the int/comparison subset: a null-free synthetic
schema). Supports fixed-length patterns (single-hop out/in/both items) — variable-length items stay
with the Python oracle.
"""
import ctypes as C
import os
import time

import numpy as np

from oracle.match_ref import Ctx, MatchContext, MatchOracle, RefDB, THRESHOLD

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(_HERE, "_build", "libdfsref.so")
MAXP, MAXA = 4, 16


class dfs_step(C.Structure):
    _fields_ = [("src", C.c_int32), ("dst", C.c_int32), ("mode", C.c_int32), ("forward", C.c_int32),
                ("nparts", C.c_int32), ("rp", C.POINTER(C.c_uint64) * MAXP), ("col", C.POINTER(C.c_uint32) * MAXP),
                ("where_bm", C.POINTER(C.c_uint64)), ("cand_bm", C.POINTER(C.c_uint64)), ("need_dedup", C.c_int32),
                ("sorted", C.c_int32)]


class dfs_plan(C.Structure):
    _fields_ = [("nsteps", C.c_int32), ("naliases", C.c_int32), ("steps", dfs_step * MAXA)]


class set_hop(C.Structure):
    _fields_ = [("src", C.c_int32), ("set_valued", C.c_int32), ("rp", C.POINTER(C.c_uint64)),
                ("col", C.POINTER(C.c_uint32)), ("where_bm", C.POINTER(C.c_uint64))]


class set_plan(C.Structure):
    _fields_ = [("nhops", C.c_int32), ("hops", set_hop * 8)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            raise ImportError("oracle C library missing: make -C oracle")
        L = C.CDLL(LIB)
        L.dfs_run.restype = C.c_int64
        L.dfs_run.argtypes = [C.POINTER(dfs_plan), C.c_int32, C.POINTER(C.c_uint32), C.c_int64, C.c_int32, C.c_int32,
                              C.POINTER(C.POINTER(C.c_uint32)), C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        L.dfs_run_ex.restype = C.c_int64
        L.dfs_run_ex.argtypes = L.dfs_run.argtypes + [C.POINTER(C.c_int32), C.c_int32, C.c_uint64,
                                                      C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        L.dfs_free.argtypes = [C.c_void_p]
        L.set_run.restype = C.c_int64
        L.set_run.argtypes = [C.POINTER(set_plan), C.c_uint32, C.POINTER(C.c_uint32), C.c_int64, C.c_int32,
                              C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        L.set_digest.restype = C.c_uint64
        L.set_digest.argtypes = [C.POINTER(C.c_int32), C.c_int32, C.c_uint64, C.c_int32]
        L.set_max_rows.restype = C.c_uint64
        L.set_max_rows.argtypes = []
        L.set_rows.restype = C.POINTER(C.c_uint32)
        L.set_rows.argtypes = [C.POINTER(C.c_uint64), C.POINTER(C.c_int32)]
        L.bfs_varlen.restype = C.c_int64
        L.bfs_varlen.argtypes = [C.POINTER(C.c_uint64), C.POINTER(C.c_uint32), C.c_uint32, C.POINTER(C.c_uint32),
                                 C.c_int64, C.c_int32, C.POINTER(C.c_uint64), C.c_int32, C.c_int32,
                                 C.POINTER(C.POINTER(C.c_uint32)), C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        L.bfs_varlen_ex.restype = C.c_int64
        L.bfs_varlen_ex.argtypes = L.bfs_varlen.argtypes + [C.c_uint64, C.POINTER(C.c_uint64)]
        _lib = L
    return _lib


MIX_H0 = 0x9E3779B97F4A7C15
RID_BASE = 11 << 48  # the synthetic Person cluster (GraphSnapshot.rmat: RID #11:v)


def _mix64(z):
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xbf58476d1ce4e5b9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94d049bb133111eb)
    return z ^ (z >> np.uint64(31))


def row_digest(rows):
    """Σ over rows of the splitmix64 chain of the row's RIDs mod 2^64 (rows: u64 [n, k], distinct) — the
    same function as the device's OMX_FLAG_DIGEST (kernels.hip k_digest)."""
    rows = np.asarray(rows, np.uint64)
    if rows.ndim == 1:
        rows = rows[:, None]
    with np.errstate(over="ignore"):
        h = np.full(rows.shape[0], MIX_H0, np.uint64)
        for c in range(rows.shape[1]):
            h = _mix64(h ^ rows[:, c])
        return int(h.sum(dtype=np.uint64)) if len(h) else 0


class CsrGraph:
    """Person/Knows graph as arrays: out CSR, in CSR (built on first use), property columns."""

    def __init__(self, rp, col, columns, trp=None, tcol=None, simple=True):
        self.V = len(rp) - 1
        self.rp = np.ascontiguousarray(rp, np.uint64)
        self.col = np.ascontiguousarray(col, np.uint32)
        self._trp = None if trp is None else np.ascontiguousarray(trp, np.uint64)
        self._tcol = None if tcol is None else np.ascontiguousarray(tcol, np.uint32)
        self.columns = columns
        self.simple = simple
        # a schema-only RefDB for the planner (class counts; no records are traversed through it)
        db = RefDB()
        db.create_class("V")
        db.create_class("E", is_edge=True)
        db.create_class("Person", "V")
        db.create_class("Knows", "E", is_edge=True)
        self._count = self.V
        db.count = lambda c: self.V if c in ("Person", "V") else 0
        self.schema = db

    def _transpose(self):
        src = np.repeat(np.arange(self.V, dtype=np.uint32), np.diff(self.rp).astype(np.int64))
        order = np.lexsort((src, self.col))
        self._tcol = np.ascontiguousarray(src[order], np.uint32)
        cnt = np.bincount(self.col, minlength=self.V)
        self._trp = np.zeros(self.V + 1, np.uint64)
        self._trp[1:] = np.cumsum(cnt)

    @property
    def trp(self):
        if self._trp is None:
            self._transpose()
        return self._trp

    @property
    def tcol(self):
        if self._tcol is None:
            self._transpose()
        return self._tcol


def np_eval(e, cols, params):
    """Vectorised restatement of Evaluator.boolean/value for the int subset (null-free columns)."""
    k = e[0]
    if k == "and":
        out = np_eval(e[1][0], cols, params)
        for x in e[1][1:]:
            out = out & np_eval(x, cols, params)
        return out
    if k == "or":
        out = np_eval(e[1][0], cols, params)
        for x in e[1][1:]:
            out = out | np_eval(x, cols, params)
        return out
    if k == "not":
        return ~np_eval(e[1], cols, params)
    if k == "paren":
        return np_eval(e[1], cols, params)
    if k == "truth":
        v = np_eval(e[1], cols, params)
        return v if isinstance(v, np.ndarray) and v.dtype == bool else np.asarray(v is True)
    if k == "cmp":
        a, b = np_eval(e[2], cols, params), np_eval(e[3], cols, params)
        op = e[1]
        return {"=": np.equal, "==": np.equal, "!=": np.not_equal, "<>": np.not_equal, "<": np.less,
                "<=": np.less_equal, ">": np.greater, ">=": np.greater_equal}[op](a, b)
    if k == "lit":
        return e[1]
    if k == "param":
        return params[e[1]]
    if k == "field":
        return cols[e[1]]
    if k == "math":
        a, b = np_eval(e[2], cols, params), np_eval(e[3], cols, params)
        return {"+": np.add, "-": np.subtract, "*": np.multiply, "%": np.mod}[e[1]](a, b)
    raise NotImplementedError("oracle C path: expression %r" % (e,))


def _bm_from_mask(mask):
    words = np.zeros((len(mask) + 63) // 64, np.uint64)
    idx = np.nonzero(mask)[0]
    np.bitwise_or.at(words, idx >> 6, np.left_shift(np.uint64(1), (idx & 63).astype(np.uint64)))
    return words


class _Steps:
    """The oracle planner's fixed-length plan over a CsrGraph (shared by the DFS and the set-based runs):
    sortEdges order, per step source/target alias, mode (0 free, 1 candidate, 2 bound), direction, CSR
    parts, target WHERE / candidate masks."""

    def __init__(self, g, query, params=None):
        mo = MatchOracle(g.schema, query)
        pmap = MatchOracle._param_map(params)
        est = mo.estimate_root_entries(Ctx(pmap))
        sorted_edges = mo.sort_edges(est)
        self.mo = mo
        self.aliases = aliases = list(mo.nodes)
        self.aidx = aidx = {a: i for i, a in enumerate(aliases)}
        prefetched = [a for a, v in est.items() if v < THRESHOLD] or [mo._next_alias(est, MatchContext())]
        if sorted_edges:
            e0, f0 = sorted_edges[0]
            root = e0.out.alias if f0 else e0.in_.alias
        else:
            root = aliases[0]
        self.root = root
        cols = g.columns
        if any(n.optional for n in mo.nodes.values()):
            raise NotImplementedError("oracle C path: optional nodes")
        if not all(e[0] == "field" and e[1] in aidx for e, _, _ in mo.st.return_items) and not any(
                t.replace(" ", "").lower() in ("$matches", "$patterns", "$paths", "$elements", "$pathelements")
                for _, _, t in mo.st.return_items):
            raise NotImplementedError("oracle C path: RETURN expressions")

        def where_mask(alias):
            w = mo.where_of(alias)
            if w is None:
                return None
            m = np_eval(w, cols, pmap)
            return np.broadcast_to(np.asarray(m, bool), (g.V,))

        def cand_mask(alias):
            m = where_mask(alias)
            return np.ones(g.V, bool) if m is None else m  # every vertex is a Person

        self.cand_mask = cand_mask
        self.steps = []
        bound = {root}
        for e, fwd in sorted_edges:
            it = e.item
            if it.multi is not None or it.filter.while_ is not None or it.filter.max_depth is not None:
                raise NotImplementedError("oracle C path: variable-length / multi items")
            s_alias, t_alias = (e.out.alias, e.in_.alias) if fwd else (e.in_.alias, e.out.alias)
            if s_alias not in bound:
                raise NotImplementedError("oracle C path: disconnected pattern")
            m = it.method.lower()
            if not fwd:
                m = {"out": "in", "in": "out", "both": "both"}[m]
            parts = {"out": lambda: [(g.rp, g.col)], "in": lambda: [(g.trp, g.tcol)],
                     "both": lambda: [(g.rp, g.col), (g.trp, g.tcol)]}[m]()
            if it.labels and not any(lab.lower() in ("knows", "e") for lab in it.labels):
                parts = []
            mode = 2 if t_alias in bound else (1 if t_alias in prefetched else 0)
            self.steps.append({"src": aidx[s_alias], "dst": aidx[t_alias], "forward": bool(fwd), "mode": mode,
                               "parts": parts, "where": where_mask(t_alias),
                               "cand": cand_mask(t_alias) if mode == 1 else None,
                               "need_dedup": len(parts) > 1 or not g.simple})
            bound.add(t_alias)
        if len(bound) != len(aliases):
            raise NotImplementedError("oracle C path: cartesian product")

    def roots(self, shard=None, root_sample=None):
        roots = np.nonzero(self.cand_mask(self.root))[0].astype(np.uint32)
        if shard is not None:  # the multi-GPU partition: root vertex v belongs to rank v % world
            roots = roots[roots % shard[1] == shard[0]]
        if root_sample is not None:
            roots = roots[:root_sample]
        return roots


def run(g, query, params=None, nthreads=1, emit=True, root_sample=None, shard=None, digest=None, distinct=None):
    """Returns dict(rows=np.uint32[n, k] (distinct, sorted; None when emit=False), aliases, bindings,
    edges, seconds, nroots). digest = RETURN aliases: every binding's projection is hashed (row_digest of
    RIDs #11:v) into r["digest"] — the digest of the result when its rows are distinct by construction.
    distinct = one RETURN alias: r["distinct"] = its distinct vertex ids (sorted), via a V-bit set."""
    sp = _Steps(g, query, params)
    aliases, aidx, root = sp.aliases, sp.aidx, sp.root
    keep = []
    plan = dfs_plan()
    plan.naliases = len(aliases)
    for i, d in enumerate(sp.steps):
        st = plan.steps[i]
        st.src, st.dst, st.forward, st.mode = d["src"], d["dst"], int(d["forward"]), d["mode"]
        st.nparts = len(d["parts"])
        for q, (rp, col) in enumerate(d["parts"]):
            st.rp[q] = rp.ctypes.data_as(C.POINTER(C.c_uint64))
            st.col[q] = col.ctypes.data_as(C.POINTER(C.c_uint32))
        st.need_dedup = int(d["need_dedup"])
        st.sorted = 1  # CsrGraph rows are sorted (the generator and the transpose sort them)
        if d["where"] is not None:
            w = _bm_from_mask(d["where"])
            keep.append(w)
            st.where_bm = w.ctypes.data_as(C.POINTER(C.c_uint64))
        if d["mode"] == 1:
            cb = _bm_from_mask(d["cand"])
            keep.append(cb)
            st.cand_bm = cb.ctypes.data_as(C.POINTER(C.c_uint64))
    plan.nsteps = len(sp.steps)
    roots = sp.roots(shard, root_sample)
    out = C.POINTER(C.c_uint32)()
    nrows = C.c_uint64()
    edges = C.c_uint64()
    proj = [aidx[a] for a in (digest or ([distinct] if distinct else []))]
    parr = (C.c_int32 * max(1, len(proj)))(*proj)
    dg = C.c_uint64()
    seen = np.zeros((g.V + 63) // 64, np.uint64) if distinct else None
    t0 = time.perf_counter()
    b = lib().dfs_run_ex(C.byref(plan), aidx[root], roots.ctypes.data_as(C.POINTER(C.c_uint32)), len(roots), nthreads,
                         int(emit), C.byref(out), C.byref(nrows), C.byref(edges), parr, len(proj), RID_BASE,
                         C.byref(dg), seen.ctypes.data_as(C.POINTER(C.c_uint64)) if seen is not None else None)
    dt = time.perf_counter() - t0
    rows = None
    if emit:
        n = nrows.value
        arr = np.ctypeslib.as_array(out, shape=(max(n, 1) * len(aliases),))[:n * len(aliases)].copy()
        lib().dfs_free(C.cast(out, C.c_void_p))
        rows = np.unique(arr.reshape(n, len(aliases)), axis=0) if n else arr.reshape(0, len(aliases))
    res = {"rows": rows, "aliases": aliases, "bindings": b, "edges": edges.value, "seconds": dt, "nroots": len(roots)}
    if digest:
        res["digest"] = dg.value
    if distinct:
        bits = np.unpackbits(seen.view(np.uint8), bitorder="little")[:g.V]
        res["distinct"] = np.nonzero(bits)[0].astype(np.uint32)
    return res


def set_run(g, query, params=None, nthreads=1, root_sample=None, digest=None, distinct=None, rows=False):
    """oracle/set_ref.c: the same bindings as run() for a chain of free hops (every step binds a new alias
    from a bound one: no closing check, no prefetched candidates), computed set-at-a-time — per hop the
    distinct sources' filtered lists once, then the rows over them (the device's algebra, on the host
    cores). Returns dict(bindings, edges, seconds, nroots, aliases[, digest][, distinct][, rows])."""
    sp = _Steps(g, query, params)
    keep = []
    plan = set_plan()
    if len(sp.steps) > 8:
        raise NotImplementedError("oracle set path: more than 8 hops")
    # column h + 1 of the row table is the h-th step's target
    colof = {sp.aidx[sp.root]: 0}
    for i, d in enumerate(sp.steps):
        if d["mode"] != 0 or len(d["parts"]) != 1:
            raise NotImplementedError("oracle set path: bound / candidate targets or several CSR parts")
        h = plan.hops[i]
        h.src = colof[d["src"]]
        colof[d["dst"]] = i + 1
        rp, col = d["parts"][0]
        h.rp = rp.ctypes.data_as(C.POINTER(C.c_uint64))
        h.col = col.ctypes.data_as(C.POINTER(C.c_uint32))
        if d["where"] is not None:
            w = _bm_from_mask(d["where"])
            keep.append(w)
            h.where_bm = w.ctypes.data_as(C.POINTER(C.c_uint64))
            h.set_valued = int(d["forward"] and d["need_dedup"])
    plan.nhops = len(sp.steps)
    roots = np.ascontiguousarray(sp.roots(None, root_sample))
    mark = None
    if distinct is not None:
        if colof[sp.aidx[distinct]] != len(sp.steps) or not sp.steps:
            raise NotImplementedError("oracle set path: a distinct column other than the last hop's")
        mark = np.zeros((g.V + 63) // 64, np.uint64)
    edges = C.c_uint64()
    t0 = time.perf_counter()
    b = lib().set_run(C.byref(plan), g.V, roots.ctypes.data_as(C.POINTER(C.c_uint32)), len(roots), int(nthreads),
                      mark.ctypes.data_as(C.POINTER(C.c_uint64)) if mark is not None else None, C.byref(edges))
    dt = time.perf_counter() - t0
    if b < 0:
        raise MemoryError("oracle/set_ref.c: a host allocation failed (the rows of %d roots)" % len(roots))
    res = {"bindings": int(b), "edges": edges.value, "seconds": dt, "nroots": len(roots), "aliases": sp.aliases,
           "max_rows": int(lib().set_max_rows())}
    if digest:
        proj = (C.c_int32 * len(digest))(*[colof[sp.aidx[a]] for a in digest])
        res["digest"] = lib().set_digest(proj, len(digest), RID_BASE, int(nthreads))
    if distinct is not None:
        bits = np.unpackbits(mark.view(np.uint8), bitorder="little")[:g.V]
        res["distinct"] = np.nonzero(bits)[0].astype(np.uint32)
    if rows:
        n, k = C.c_uint64(), C.c_int32()
        p = lib().set_rows(C.byref(n), C.byref(k))
        arr = np.ctypeslib.as_array(p, shape=(max(1, n.value * k.value),))[:n.value * k.value].reshape(-1, k.value)
        order = [colof[sp.aidx[a]] for a in sp.aliases]
        res["rows"] = arr[:, order].copy()
    return res


def bfs_varlen(rp, col, roots, max_depth=-1, where_mask=None, nthreads=1, emit=True):
    """oracle/bfs_ref.c: variable-length item with depth-free WHERE and a depth-only while (the result
    is the BFS ball of radius max_depth; -1 = unbounded). Returns dict(pairs=np.uint32[n, 2] of
    (root index, v) or None, n, edges, seconds, digest = row_digest of the (RID(root), RID(v)) rows)."""
    rp = np.ascontiguousarray(rp, np.uint64)
    col = np.ascontiguousarray(col, np.uint32)
    roots = np.ascontiguousarray(roots, np.uint32)
    V = len(rp) - 1
    wb = _bm_from_mask(np.asarray(where_mask, bool)) if where_mask is not None else None
    out = C.POINTER(C.c_uint32)()
    npairs = C.c_uint64()
    edges = C.c_uint64()
    t0 = time.perf_counter()
    dg = C.c_uint64()
    n = lib().bfs_varlen_ex(rp.ctypes.data_as(C.POINTER(C.c_uint64)), col.ctypes.data_as(C.POINTER(C.c_uint32)), V,
                            roots.ctypes.data_as(C.POINTER(C.c_uint32)), len(roots), int(max_depth),
                            wb.ctypes.data_as(C.POINTER(C.c_uint64)) if wb is not None else None, int(nthreads),
                            int(emit), C.byref(out), C.byref(npairs), C.byref(edges), RID_BASE, C.byref(dg))
    dt = time.perf_counter() - t0
    pairs = None
    if emit:
        pairs = np.ctypeslib.as_array(out, shape=(max(1, npairs.value) * 2,))[:npairs.value * 2].reshape(-1, 2).copy()
        lib().dfs_free(C.cast(out, C.c_void_p))
    return {"pairs": pairs, "n": int(n), "edges": int(edges.value), "seconds": dt, "digest": dg.value}
