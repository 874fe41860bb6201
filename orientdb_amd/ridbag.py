"""Ridbag ingest: the vertices' serialized out_<L> / in_<L> fields → a CSR, decoded on the device.

Mirrors what building a snapshot from stored records needs instead of iterating every vertex's
ORidBag (C/db/record/ridbag/ORidBag.java:160 rawIterator) in Java: the record bytes of the bags go to
the device as they are (ORidBag.toStream, ORidBag.java:198-276; OEmbeddedRidBag.serialize,
.../ridbag/embedded/OEmbeddedRidBag.java:424-460) and come back as row pointers + dense vertex ids
(include/omx/match.h omx_ridbag_decode_csr).
"""
import ctypes as C

import numpy as np

from . import _native as N


def _u64p(a):
    return a.ctypes.data_as(C.POINTER(C.c_uint64)) if a is not None else None


def decode_ridbags(streams, vertex_rids, edge_rids=None, edge_targets=None, device=0, files=None,
                   page_size=65536, entry_rids=False):
    """streams: one bytes object per vertex (b"" = the vertex has no such field), in dense vertex order.
    vertex_rids: packed RID of every vertex. edge_rids / edge_targets: for regular (non-lightweight)
    edges, every edge record's RID and the packed RID of its opposite vertex. files: {fileId: pages
    (bytes-like, n × page_size)} of the SBTree collection files that SBTree-bonsai bags point into
    (None: embedded bags only). Returns (row_ptr u64[V+1], col u32[E]) with each bag's iteration order;
    entry_rids (edge records only): + the edge record RID of every entry (omx_ridbag_decode_edges), the
    edge_rids of an edge-records snapshot."""
    V = len(streams)
    offs = np.zeros(V + 1, np.uint64)
    offs[1:] = np.cumsum([len(b) for b in streams], dtype=np.uint64)
    blob = b"".join(streams)
    return decode_ridbag_blob(blob, offs, vertex_rids, edge_rids, edge_targets, device, files, page_size, entry_rids)


def decode_ridbag_blob(blob, offsets, vertex_rids, edge_rids=None, edge_targets=None, device=0, files=None,
                       page_size=65536, entry_rids=False):
    """The same over one concatenated byte string and its offsets[V+1]."""
    offs = np.ascontiguousarray(offsets, np.uint64)
    V = len(offs) - 1
    vr = np.ascontiguousarray(vertex_rids, np.uint64)
    if len(vr) != V:
        raise ValueError("vertex_rids must have one RID per stream")
    er = np.ascontiguousarray(edge_rids, np.uint64) if edge_rids is not None else None
    et = np.ascontiguousarray(edge_targets, np.uint64) if edge_targets is not None else None
    ne = len(er) if er is not None else 0
    buf = np.frombuffer(blob, np.uint8) if len(blob) else np.zeros(1, np.uint8)
    rp = np.zeros(V + 1, np.uint64)
    n = C.c_uint64()
    L = N.lib()
    args = [device, buf.ctypes.data_as(C.c_void_p), len(blob), _u64p(offs), V, _u64p(vr), _u64p(er), _u64p(et), ne]
    if entry_rids and er is None:
        raise ValueError("entry_rids needs the edge records (edge_rids, edge_targets)")
    if files is None and not entry_rids:
        fn, extra = L.omx_ridbag_decode_csr, []
    elif files is None:
        fn, extra = L.omx_ridbag_decode_edges, [None, 0, page_size]
    else:
        keep = [np.frombuffer(bytes(p), np.uint8) if len(p) else np.zeros(1, np.uint8) for p in files.values()]
        recs = (N.omx_bonsai_file * max(1, len(files)))()
        for i, (fid, pages) in enumerate(files.items()):
            if len(pages) % page_size:
                raise ValueError("collection file %d is not a whole number of pages" % fid)
            recs[i].file_id = int(fid)
            recs[i].pages = keep[i].ctypes.data_as(C.c_void_p)
            recs[i].n_pages = len(pages) // page_size
        fn = L.omx_ridbag_decode_edges if entry_rids else L.omx_ridbag_decode_csr_ex
        extra = [C.cast(recs, C.c_void_p), len(files), page_size]
    if entry_rids:
        N.check(fn(*args, *extra, _u64p(rp), None, None, C.byref(n)))
        col = np.zeros(max(n.value, 1), np.uint32)
        ent = np.zeros(max(n.value, 1), np.uint64)
        N.check(fn(*args, *extra, _u64p(rp), col.ctypes.data_as(C.POINTER(C.c_uint32)), _u64p(ent), C.byref(n)))
        return rp, col[:n.value], ent[:n.value]
    N.check(fn(*args, *extra, _u64p(rp), None, C.byref(n)))
    col = np.zeros(max(n.value, 1), np.uint32)
    N.check(fn(*args, *extra, _u64p(rp), col.ctypes.data_as(C.POINTER(C.c_uint32)), C.byref(n)))
    return rp, col[:n.value]
