"""HBM snapshot of a database for the MATCH path (omx_graph_create).

A snapshot holds what the reference's MATCH reads record by record (SURVEY.md §8(a) a11–a13):
per edge class the out_/in_ ridbags of every vertex as CSR, every vertex's class and RID, and one
column per property. It is built once and shared read-only by every statement executed on it.
"""
import ctypes as C
import os
import json

import numpy as np

from . import _native as N

RID_POS_BITS = 48


def pack_rid(cluster, position):
    return (int(cluster) << RID_POS_BITS) | int(position)


def unpack_rid(r):
    r = int(r)
    return r >> RID_POS_BITS, r & ((1 << RID_POS_BITS) - 1)


def _ptr(a, ctype):
    return a.ctypes.data_as(C.POINTER(ctype)) if a is not None else None


class GraphSnapshot:
    """One omx_graph. `classes` = list of (name, superclass index or -1, is_edge, cluster id);
    `edge_sets` = list of dicts {cls, out_rp, out_col[, in_rp, in_col][, edge_rids[, in_edge_index]]} (numpy
    u64/u32; edge_rids: the edge records behind the out entries, on every set or none);
    `properties` = list of dicts {name, type, values[, present][, dict]};
    `indexes` = list of (class index, property name, unique);
    `edge_properties` = fields of the edge records (as `properties`, indexed by the sets' out entries one
    after another)."""

    def __init__(self, n_vertices, classes, vertex_class, rids, edge_sets, properties=(), indexes=(), device=0,
                 part=None, edge_properties=()):
        """part = (lo, hi): a 1-D partition holding the CSR rows of vertices [lo, hi) only (local row
        pointers of hi − lo + 1 entries; the in CSR is required); see include/omx/match.h."""
        L = N.lib()
        self.V = int(n_vertices)
        self.classes = list(classes)
        self.class_names = [c[0] for c in self.classes]
        self.vertex_class = np.ascontiguousarray(vertex_class, dtype=np.uint16)
        self.rids = np.ascontiguousarray(rids, dtype=np.uint64)
        self.device = device
        keep = []
        cls_arr = (N.omx_class_desc * len(self.classes))()
        for i, (name, sup, is_edge, cluster) in enumerate(self.classes):
            b = name.encode()
            keep.append(b)
            cls_arr[i] = N.omx_class_desc(b, sup, int(is_edge), cluster)
        es_arr = (N.omx_edge_set_desc * max(1, len(edge_sets)))()
        for i, es in enumerate(edge_sets):
            orp = np.ascontiguousarray(es["out_rp"], dtype=np.uint64)
            ocol = np.ascontiguousarray(es["out_col"], dtype=np.uint32)
            irp = es.get("in_rp")
            icol = es.get("in_col")
            irp = None if irp is None else np.ascontiguousarray(irp, dtype=np.uint64)
            icol = None if icol is None else np.ascontiguousarray(icol, dtype=np.uint32)
            erid = es.get("edge_rids")
            erid = None if erid is None else np.ascontiguousarray(erid, dtype=np.uint64)
            eix = es.get("in_edge_index")
            eix = None if eix is None else np.ascontiguousarray(eix, dtype=np.uint64)
            keep += [orp, ocol, irp, icol, erid, eix]
            es_arr[i] = N.omx_edge_set_desc(es["cls"], int(orp[-1]), _ptr(orp, C.c_uint64), _ptr(ocol, C.c_uint32),
                                            _ptr(irp, C.c_uint64), _ptr(icol, C.c_uint32),
                                            int(irp[-1]) if irp is not None else 0, _ptr(erid, C.c_uint64),
                                            _ptr(eix, C.c_uint64))
        pr_arr = _property_array(properties, keep)
        epr_arr = _property_array(edge_properties, keep)
        ix_arr = (N.omx_index_desc * max(1, len(indexes)))()
        for i, (ci, prop, unique) in enumerate(indexes):
            b = prop.encode()
            keep.append(b)
            ix_arr[i] = N.omx_index_desc(ci, b, int(unique))
        self.part = (0, self.V) if part is None else (int(part[0]), int(part[1]))
        desc = N.omx_graph_desc(self.V, len(self.classes), cls_arr, _ptr(self.vertex_class, C.c_uint16),
                                _ptr(self.rids, C.c_uint64), len(edge_sets), es_arr, len(properties), pr_arr,
                                len(indexes), ix_arr, device, *((0, 0) if part is None else self.part),
                                len(edge_properties), epr_arr)
        h = C.c_void_p()
        N.check(L.omx_graph_create(C.byref(desc), C.byref(h)))
        self._h = h
        self.properties = {p["name"]: p for p in properties}

    @property
    def handle(self):
        if self._h is None:
            raise RuntimeError("graph snapshot closed")
        return self._h

    def class_count(self, name):
        n = C.c_uint64()
        N.check(N.lib().omx_graph_class_count(self.handle, name.encode(), C.byref(n)))
        return n.value

    def device_bytes(self):
        return N.lib().omx_graph_device_bytes(self.handle)

    def close(self):
        if getattr(self, "_h", None) is not None:
            N.lib().omx_graph_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---------------------------------------------------------------------------------------------
    @classmethod
    def from_blob(cls, buf):
        """omx_graph_create_blob: a snapshot from one pointer-free buffer (include/omx/match.h), as a
        Java builder fills it (buf: an 8-byte aligned numpy array)."""
        L = N.lib()
        h = C.c_void_p()
        N.check(L.omx_graph_create_blob(buf.ctypes.data_as(C.c_void_p), buf.nbytes, C.byref(h)))
        g = cls.__new__(cls)
        g._h = h
        g.V = int(np.frombuffer(buf.tobytes()[8:12], np.uint32)[0])
        g.part = (0, g.V)
        return g

    @classmethod
    def from_records(cls, db, device=0, edge_records=False):
        """Snapshot of a record-level description (the JSON of tests/golden/make_match_test_db.py):
        classes in creation order, one cluster per class (ids from 11), vertices in insertion order.
        edge_records: the edges as records (RID #cluster:rank within the class, fields from each edge's
        "props"), so MATCH can bind edge nodes; otherwise lightweight adjacency."""
        a = records_arrays(db, edge_records)
        g = cls(*a[:7], device, None, a[7] if edge_records else ())
        g.records = db
        return g



    @classmethod
    def person_knows(cls, rp, col, seed, device=0, keep_csr=False):
        """Person/Knows snapshot over a given out-CSR (SURVEY.md §8(d) schema): vertices of class Person
        (one cluster → RID #11:v), edge class Knows, properties uid (int64 = v) and age (int32 uniform
        [0,100) from a seeded splitmix64)."""
        V = len(rp) - 1
        classes = [("V", -1, False, 9), ("E", -1, True, 10), ("Person", 0, False, 11), ("Knows", 1, True, 12)]
        vclass = np.full(V, 2, np.uint16)
        rids = (np.uint64(11) << np.uint64(RID_POS_BITS)) | np.arange(V, dtype=np.uint64)
        props = [{"name": "uid", "type": N.OMX_PROP_INT64, "values": np.arange(V, dtype=np.int64)},
                 {"name": "age", "type": N.OMX_PROP_INT32, "values": synthetic_int_column(V, seed ^ 0xA9E, 100)}]
        g = cls(V, classes, vclass, rids, [{"cls": 3, "out_rp": rp, "out_col": col}], props, [], device)
        g.n_edges = int(rp[-1])
        if keep_csr:
            g.csr = (rp, col)
        g.age = props[1]["values"]
        return g

    @classmethod
    def ldbc_like(cls, n_persons=70000, target_edges=2_000_000, seed=10, device=0, keep_csr=False):
        """LDBC-SNB-like SF10 Knows graph (configs[3]; generator in gen.cpp) with the Person/Knows schema."""
        rp, col = ldbc_csr(n_persons, target_edges, seed)
        return cls.person_knows(rp, col, seed, device, keep_csr)

    @classmethod
    def rmat(cls, scale, edge_factor=16, seed=None, simple=True, device=0, keep_csr=False, partition=None,
             edge_records=False):
        """Synthetic Person/Knows graph: Graph500 RMAT, vertices of class Person
        (one cluster → RID #11:v), edge class Knows, properties uid (int64 = v) and age (int32 uniform
        [0,100) from a seeded splitmix64). partition = (rank, world): the 1-D partition of that rank
        (rows of the vertices [rank·B, (rank+1)·B), B = ⌈V/world⌉; generated without the other rows).
        edge_records: the Knows edges as records — RID #12:i for out-CSR entry i, field `w` (int32 uniform
        [0,100) from a seeded splitmix64) — so MATCH can bind and filter edge nodes (unpartitioned only)."""
        seed = scale if seed is None else seed
        V = 1 << scale
        part = None
        if partition is None:
            rp, col = rmat_csr(scale, edge_factor, seed, simple, device=device)
            es = {"cls": 3, "out_rp": rp, "out_col": col}
        else:
            part = partition_range(V, *partition)
            rp, col, irp, icol = rmat_partition(scale, part[0], part[1], edge_factor, seed, simple, device=device)
            es = {"cls": 3, "out_rp": rp, "out_col": col, "in_rp": irp, "in_col": icol}
        classes = [("V", -1, False, 9), ("E", -1, True, 10), ("Person", 0, False, 11), ("Knows", 1, True, 12)]
        vclass = np.full(V, 2, np.uint16)
        rids = (np.uint64(11) << np.uint64(RID_POS_BITS)) | np.arange(V, dtype=np.uint64)
        props = [{"name": "uid", "type": N.OMX_PROP_INT64, "values": np.arange(V, dtype=np.int64)},
                 {"name": "age", "type": N.OMX_PROP_INT32, "values": synthetic_int_column(V, seed ^ 0xA9E, 100)}]
        eprops = ()
        if edge_records:
            if partition is not None:
                raise ValueError("edge records on a partitioned snapshot are not supported")
            ne = int(rp[-1])
            es["edge_rids"] = (np.uint64(12) << np.uint64(RID_POS_BITS)) | np.arange(ne, dtype=np.uint64)
            eprops = [{"name": "w", "type": N.OMX_PROP_INT32, "values": synthetic_int_column(ne, seed ^ 0xED6E, 100)}]
        g = cls(V, classes, vclass, rids, [es], props, [], device, part, eprops)
        if edge_records:
            g.w = eprops[0]["values"]
        g.scale = scale
        g.n_edges = int(rp[-1])
        if keep_csr:
            g.csr = (rp, col)
        g.age = props[1]["values"]
        return g



def _property_array(properties, keep):
    arr = (N.omx_property_desc * max(1, len(properties)))()
    for i, p in enumerate(properties):
        t = p["type"]
        dt = {N.OMX_PROP_INT32: np.int32, N.OMX_PROP_INT64: np.int64, N.OMX_PROP_DOUBLE: np.float64,
              N.OMX_PROP_STRING: np.int32, N.OMX_PROP_BOOL: np.int32}[t]
        vals = np.ascontiguousarray(p["values"], dtype=dt)
        pres = p.get("present")
        pres = None if pres is None else np.ascontiguousarray(pres, dtype=np.uint8)
        d = p.get("dict") or []
        dict_arr = (C.c_char_p * max(1, len(d)))(*[s.encode() for s in d]) if d else None
        nb = p["name"].encode()
        keep += [vals, pres, dict_arr, nb]
        arr[i] = N.omx_property_desc(nb, t, vals.ctypes.data_as(C.c_void_p), _ptr(pres, C.c_uint8),
                                     len(d), C.cast(dict_arr, C.POINTER(C.c_char_p)) if dict_arr else None)
    return arr


def _columns(recs):
    """One property column per field name over the records' "props" dicts (absent → not present)."""
    fields = []
    for rec in recs:
        for k in rec.get("props", {}):
            if k not in fields:
                fields.append(k)
    props = []
    for f in fields:
        vals = [rec.get("props", {}).get(f) for rec in recs]
        present = np.array([x is not None for x in vals], np.uint8)
        nonnull = [x for x in vals if x is not None]
        if all(isinstance(x, str) for x in nonnull):
            d = sorted(set(nonnull), key=lambda s: s.encode())
            code = {s: i for i, s in enumerate(d)}
            col = np.array([code[x] if x is not None else -1 for x in vals], np.int32)
            props.append({"name": f, "type": N.OMX_PROP_STRING, "values": col, "present": present, "dict": d})
        elif all(isinstance(x, bool) for x in nonnull):
            col = np.array([int(x) if x is not None else 0 for x in vals], np.int32)
            props.append({"name": f, "type": N.OMX_PROP_BOOL, "values": col, "present": present})
        elif all(isinstance(x, int) and not isinstance(x, bool) for x in nonnull):
            col = np.array([x if x is not None else 0 for x in vals], np.int64)
            props.append({"name": f, "type": N.OMX_PROP_INT64, "values": col, "present": present})
        else:
            col = np.array([float(x) if x is not None else 0.0 for x in vals], np.float64)
            props.append({"name": f, "type": N.OMX_PROP_DOUBLE, "values": col, "present": present})
    return props


def records_arrays(db, edge_records=False):
    """(V, classes, vertex_class, rids, edge_sets, properties, indexes) of a record-level description
    (GraphSnapshot.from_records); edge_records: + the edge records (edge_rids per set) and an 8th item,
    the edge records' property columns."""
    if isinstance(db, str):
        with open(db) as f:
            db = json.load(f)
    names = [c["name"] for c in db["classes"]]
    classes = []
    for i, c in enumerate(db["classes"]):
        sup = names.index(c["superclass"]) if c["superclass"] is not None else -1
        classes.append((c["name"], sup, bool(c["is_edge"]), 11 + i))
    V = len(db["vertices"])
    vclass = np.zeros(V, np.uint16)
    rids = np.zeros(V, np.uint64)
    per_class = {}
    for v, rec in enumerate(db["vertices"]):
        ci = names.index(rec["class"])
        vclass[v] = ci
        pos = per_class.get(ci, 0)
        per_class[ci] = pos + 1
        rids[v] = pack_rid(classes[ci][3], pos)
    # adjacency: one CSR per edge class, rows in insertion order (ridbag order)
    edge_sets = []
    edge_recs = []  # the edge records in edge-id order (the sets' out entries one after another)
    for ci, (name, _, is_edge, cluster) in enumerate(classes):
        if not is_edge:
            continue
        recs = [e for e in db["edges"] if e["class"] == name]  # rank within the class = RID position
        if not recs:
            continue
        src = np.array([e["out"] for e in recs], np.int64)
        dst = np.array([e["in"] for e in recs], np.uint32)
        order = np.argsort(src, kind="stable")
        rp = np.zeros(V + 1, np.uint64)
        np.add.at(rp, src + 1, 1)
        rp = np.cumsum(rp).astype(np.uint64)
        es = {"cls": ci, "out_rp": rp, "out_col": dst[order]}
        if edge_records:
            es["edge_rids"] = (np.uint64(cluster) << np.uint64(RID_POS_BITS)) | order.astype(np.uint64)
            edge_recs += [recs[k] for k in order]
        edge_sets.append(es)
    props = _columns(db["vertices"])
    indexes = [(names.index(ix["class"]), ix["property"], bool(ix["unique"])) for ix in db.get("indexes", [])]
    if edge_records:
        return V, classes, vclass, rids, edge_sets, props, indexes, _columns(edge_recs)
    return V, classes, vclass, rids, edge_sets, props, indexes


def ldbc_csr(n_persons=70000, target_edges=2_000_000, seed=10):
    """(row_ptr u64[V+1], col u32[E]) of the LDBC-SNB-like Knows generator in libomx (configs[3])."""
    L = N.lib()
    prp = C.POINTER(C.c_uint64)()
    pcol = C.POINTER(C.c_uint32)()
    ne = C.c_uint64()
    N.check(L.omx_ldbc_knows_generate(n_persons, target_edges, seed, C.byref(prp), C.byref(pcol), C.byref(ne)))
    rp = np.ctypeslib.as_array(prp, shape=(n_persons + 1,)).copy()
    col = np.ctypeslib.as_array(pcol, shape=(max(1, ne.value),))[:ne.value].copy()
    L.omx_host_free(C.cast(prp, C.c_void_p))
    L.omx_host_free(C.cast(pcol, C.c_void_p))
    return rp, col


def _gen_device(device):
    """Device for the RMAT generator: the snapshot's GPU (gen.hip: draws + radix sort, the same arrays as
    the host generator gen.cpp), or None for the host generator (CPU snapshots, OMX_GEN_HOST=1)."""
    if device is None or device < 0 or os.environ.get("OMX_GEN_HOST") == "1":
        return None
    return device


def rmat_csr(scale, edge_factor=16, seed=None, simple=True, device=None):
    """(row_ptr u64[V+1], col u32[E]) of the deterministic RMAT generator in libomx (built on `device`
    when one is given)."""
    L = N.lib()
    seed = scale if seed is None else seed
    prp = C.POINTER(C.c_uint64)()
    pcol = C.POINTER(C.c_uint32)()
    ne = C.c_uint64()
    dev = _gen_device(device)
    if dev is None:
        N.check(L.omx_rmat_generate(scale, edge_factor, seed, int(simple), C.byref(prp), C.byref(pcol), C.byref(ne)))
    else:
        N.check(L.omx_rmat_generate_dev(dev, scale, edge_factor, seed, int(simple), C.byref(prp), C.byref(pcol),
                                        C.byref(ne)))
    V = 1 << scale
    rp = np.ctypeslib.as_array(prp, shape=(V + 1,)).copy()
    col = np.ctypeslib.as_array(pcol, shape=(max(1, ne.value),))[:ne.value].copy()
    L.omx_host_free(C.cast(prp, C.c_void_p))
    L.omx_host_free(C.cast(pcol, C.c_void_p))
    return rp, col


def partition_range(V, rank, world):
    """Rows [lo, hi) of rank `rank` under the block partition of include/omx/match.h (B = ⌈V/world⌉)."""
    b = -(-int(V) // int(world))
    return min(V, rank * b), min(V, (rank + 1) * b)


def rmat_partition(scale, lo, hi, edge_factor=16, seed=None, simple=True, device=None):
    """(out_rp, out_col, in_rp, in_col) of the RMAT rows [lo, hi) (local row pointers)."""
    L = N.lib()
    seed = scale if seed is None else seed
    orp, ocol, irp, icol = C.POINTER(C.c_uint64)(), C.POINTER(C.c_uint32)(), C.POINTER(C.c_uint64)(), C.POINTER(C.c_uint32)()
    no, ni = C.c_uint64(), C.c_uint64()
    dev = _gen_device(device)
    if dev is None:
        N.check(L.omx_rmat_generate_part(scale, edge_factor, seed, int(simple), lo, hi, C.byref(orp), C.byref(ocol),
                                         C.byref(no), C.byref(irp), C.byref(icol), C.byref(ni)))
    else:
        N.check(L.omx_rmat_generate_part_dev(dev, scale, edge_factor, seed, int(simple), lo, hi, C.byref(orp),
                                             C.byref(ocol), C.byref(no), C.byref(irp), C.byref(icol), C.byref(ni)))
    n = hi - lo
    out = (np.ctypeslib.as_array(orp, shape=(n + 1,)).copy(),
           np.ctypeslib.as_array(ocol, shape=(max(1, no.value),))[:no.value].copy(),
           np.ctypeslib.as_array(irp, shape=(n + 1,)).copy(),
           np.ctypeslib.as_array(icol, shape=(max(1, ni.value),))[:ni.value].copy())
    for p in (orp, ocol, irp, icol):
        L.omx_host_free(C.cast(p, C.c_void_p))
    return out


def csr_transpose(V, rp, col):
    L = N.lib()
    rp = np.ascontiguousarray(rp, np.uint64)
    col = np.ascontiguousarray(col, np.uint32)
    prp = C.POINTER(C.c_uint64)()
    pcol = C.POINTER(C.c_uint32)()
    N.check(L.omx_csr_transpose(V, _ptr(rp, C.c_uint64), _ptr(col, C.c_uint32), C.byref(prp), C.byref(pcol)))
    E = int(rp[-1])
    trp = np.ctypeslib.as_array(prp, shape=(V + 1,)).copy()
    tcol = np.ctypeslib.as_array(pcol, shape=(max(1, E),))[:E].copy()
    L.omx_host_free(C.cast(prp, C.c_void_p))
    L.omx_host_free(C.cast(pcol, C.c_void_p))
    return trp, tcol


def synthetic_int_column(V, seed, modulo):
    L = N.lib()
    p = C.POINTER(C.c_int32)()
    N.check(L.omx_synthetic_int_column(V, seed, modulo, C.byref(p)))
    out = np.ctypeslib.as_array(p, shape=(max(1, V),))[:V].copy()
    L.omx_host_free(C.cast(p, C.c_void_p))
    return out
