"""The pointer-free buffers of include/omx/match.h (omx_graph_create_blob / omx_execute_packed), laid
out byte by byte the way a Java snapshot builder fills a direct ByteBuffer: a header at offset 0,
fixed-size records, every pointer replaced by a byte offset into the same buffer (0 = none), arrays
naturally aligned, strings NUL-terminated UTF-8. Test infrastructure: nothing in the product imports it.
"""
import struct

import numpy as np

MAGIC, VERSION = 0x47584D4F, 2


class _Buf:
    def __init__(self, header_size):
        self.b = bytearray(header_size)

    def put(self, data, align=8):
        while len(self.b) % align:
            self.b.append(0)
        off = len(self.b)
        self.b += data
        return off

    def put_str(self, s):
        return self.put(s.encode("utf-8") + b"\0", 1)

    def put_array(self, a, dtype):
        a = np.ascontiguousarray(a, dtype)
        return self.put(a.tobytes(), a.dtype.itemsize) if a.size else 0


def _props(B, properties):
    prec = b""
    for p in properties:
        t = p["type"]
        dt = {1: np.int32, 2: np.int64, 3: np.float64, 4: np.int32, 5: np.int32}[t]
        v_off = B.put_array(p["values"], dt)
        pres = p.get("present")
        pr_off = B.put_array(pres, np.uint8) if pres is not None else 0
        d = p.get("dict") or []
        d_off = B.put(struct.pack("<%dQ" % len(d), *[B.put_str(s) for s in d])) if d else 0
        prec += struct.pack("<QiiQQQ", B.put_str(p["name"]), t, len(d), v_off, pr_off, d_off)
    return B.put(prec) if prec else 0


def graph_blob(n_vertices, classes, vertex_class, rids, edge_sets, properties=(), indexes=(), device=0, part=None,
               edge_properties=(), version=VERSION):
    """Arguments as GraphSnapshot(...) takes them; returns (bytes, numpy u64 buffer keeping it 8-aligned).
    version 1: the 88-byte header without edge records."""
    B = _Buf(112 if version >= 2 else 88)
    crec = b""
    for name, sup, is_edge, cluster in classes:
        crec += struct.pack("<Qiiii", B.put_str(name), sup, int(is_edge), cluster, 0)
    classes_off = B.put(crec)
    vc_off = B.put_array(vertex_class, np.uint16)
    rid_off = B.put_array(rids, np.uint64)
    erec = b""
    for es in edge_sets:
        orp = np.asarray(es["out_rp"], np.uint64)
        irp = es.get("in_rp")
        o_rp, o_col = B.put_array(orp, np.uint64), B.put_array(es["out_col"], np.uint32)
        i_rp = B.put_array(irp, np.uint64) if irp is not None else 0
        i_col = B.put_array(es["in_col"], np.uint32) if irp is not None else 0
        n_in = int(np.asarray(irp)[-1]) if irp is not None else 0
        erec += struct.pack("<iiQQQQQQ", es["cls"], 0, int(orp[-1]), o_rp, o_col, i_rp, i_col, n_in)
    es_off = B.put(erec) if erec else 0
    xr_off = 0
    if edge_sets and all(es.get("edge_rids") is not None for es in edge_sets):
        xrec = b""
        for es in edge_sets:
            eix = es.get("in_edge_index")
            xrec += struct.pack("<QQ", B.put_array(es["edge_rids"], np.uint64),
                                B.put_array(eix, np.uint64) if eix is not None else 0)
        xr_off = B.put(xrec)
    pr_off = _props(B, properties)
    epr_off = _props(B, edge_properties)
    irec = b"".join(struct.pack("<Qii", B.put_str(prop), ci, int(u)) for ci, prop, u in indexes)
    ix_off = B.put(irec) if irec else 0
    lo, hi = part if part is not None else (0, 0)
    struct.pack_into("<IIIiiiiiIIQQQQQQ", B.b, 0, MAGIC, version, n_vertices, len(classes), len(edge_sets),
                     len(properties), len(indexes), device, lo, hi, classes_off, vc_off, rid_off, es_off, pr_off, ix_off)
    if version >= 2:
        struct.pack_into("<QiiQ", B.b, 88, xr_off, len(edge_properties), 0, epr_off)
    while len(B.b) % 8:
        B.b.append(0)
    return np.frombuffer(bytes(B.b), np.uint64).copy()


def param_blob(args=(), named=None):
    """uint32 n, uint32 0, omx_param_rec[n], strings (positional args, then named)."""
    items = [(i, None, a) for i, a in enumerate(args)] + [(0, k, a) for k, a in (named or {}).items()]
    n = len(items)
    B = _Buf(8 + 40 * n)
    recs = []
    for idx, name, a in items:
        name_off = B.put_str(name) if name else 0
        t, i, d, s_off = 0, 0, 0.0, 0
        if a is None:
            t = 0
        elif isinstance(a, bool):
            t, i = 4, int(a)
        elif isinstance(a, int):
            t, i = 1, a
        elif isinstance(a, float):
            t, d = 2, a
        else:
            t, s_off = 3, B.put_str(str(a))
        recs.append(struct.pack("<iiqdQQ", t, idx, i, d, name_off, s_off))
    struct.pack_into("<II", B.b, 0, n, 0)
    for k, r in enumerate(recs):
        B.b[8 + 40 * k: 48 + 40 * k] = r
    while len(B.b) % 8:
        B.b.append(0)
    return np.frombuffer(bytes(B.b), np.uint64).copy()
