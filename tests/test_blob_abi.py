"""The pointer-free boundary (include/omx/match.h omx_graph_create_blob / omx_execute_packed): the
buffers are built byte by byte the way a Java snapshot builder fills a direct ByteBuffer
(tests/blob_builder.py), and must describe exactly the snapshot the pointer descriptor does."""
import ctypes as C

import numpy as np
import pytest

from tests.blob_builder import graph_blob, param_blob
from tests.known_answers import KNOWN


@pytest.fixture(scope="module")
def blob_graphs(match_test_db_json):
    import orientdb_amd as o
    from orientdb_amd.graph import records_arrays
    arrays = records_arrays(match_test_db_json)
    ref = o.GraphSnapshot(*arrays, device=-1)
    buf = graph_blob(*arrays, device=-1)
    return ref, o.GraphSnapshot.from_blob(buf), buf


def test_blob_snapshot_equals_pointer_snapshot(blob_graphs):
    ref, g, _ = blob_graphs
    for cls in ("V", "E", "Person", "Employee", "TriangleV", "IndexedVertex"):
        assert g.class_count(cls) == ref.class_count(cls)


@pytest.mark.parametrize("case", KNOWN[::3], ids=[k[0] for k in KNOWN[::3]])
def test_blob_snapshot_plans_like_pointer_snapshot(blob_graphs, case):
    import orientdb_amd as o
    ref, g, _ = blob_graphs
    st = o.OMatchStatement(case[2])
    assert st.explain(g, *(case[3] or [])) == st.explain(ref, *(case[3] or []))


def _create(buf, size=None):
    import orientdb_amd as o
    h = C.c_void_p()
    rc = o._native.lib().omx_graph_create_blob(buf.ctypes.data_as(C.c_void_p), buf.nbytes if size is None else size,
                                               C.byref(h))
    if rc == 0:
        o._native.lib().omx_graph_destroy(h)
    return rc


def test_blob_rejects_bad_buffers(blob_graphs):
    import orientdb_amd as o
    _, _, buf = blob_graphs
    assert _create(buf) == 0
    bad = buf.copy()
    bad.view(np.uint32)[0] = 0xDEAD  # magic
    assert _create(bad) == o._native.OMX_E_INVALID
    assert _create(buf, size=64) == o._native.OMX_E_INVALID  # truncated header
    assert _create(buf, size=buf.nbytes // 2) == o._native.OMX_E_INVALID  # arrays past the end
    bad = buf.copy()
    bad.view(np.uint64)[6] += 1  # classes_off (header word 6) misaligned
    assert _create(bad) == o._native.OMX_E_INVALID
    bad = buf.copy()
    bad.view(np.uint64)[7] = buf.nbytes * 4  # vertex_class_off out of range
    assert _create(bad) == o._native.OMX_E_INVALID


def _edge_set0(buf):
    """(n_vertices, out_row_ptr offset, out_col offset, in_col offset) of the first edge-set record."""
    raw = buf.view(np.uint8)
    V = int(raw[8:12].view(np.uint32)[0])
    es_off = int(buf[8])  # header word 8
    rec = raw[es_off:es_off + 56].view(np.uint64)
    return V, int(rec[2]), int(rec[3]), int(rec[5]), int(rec[1])


def test_blob_rejects_bad_contents(blob_graphs):
    """Contents, not only extents: a column id >= n_vertices (out or in) or a decreasing row pointer fails
    with OMX_E_INVALID at create time instead of reaching the kernels (capi.cpp check_csr)."""
    import orientdb_amd as o
    _, _, buf = blob_graphs
    V, o_rp, o_col, i_col, n_e = _edge_set0(buf)
    assert n_e > 0
    raw = buf.view(np.uint8)
    bad = buf.copy()
    bad.view(np.uint8)[o_col:o_col + 4].view(np.uint32)[0] = V  # out-of-range neighbour
    assert _create(bad) == o._native.OMX_E_INVALID
    bad = buf.copy()
    bad.view(np.uint8)[i_col + 4 * (n_e - 1):i_col + 4 * n_e].view(np.uint32)[0] = 0xFFFFFFF0
    assert _create(bad) == o._native.OMX_E_INVALID
    rp = raw[o_rp:o_rp + 8 * (V + 1)].view(np.uint64)
    i = int(np.nonzero(np.diff(rp.astype(np.int64)) > 0)[0][0])  # rp[i] < rp[i + 1]
    bad = buf.copy()
    brp = bad.view(np.uint8)[o_rp:o_rp + 8 * (V + 1)].view(np.uint64)
    brp[i + 1] = brp[i + 2] + 1 if i + 2 <= V else brp[i + 1]  # rp[i+1] > rp[i+2]
    brp[i] = brp[i + 1] + 5  # rp[i] > rp[i+1]
    assert _create(bad) == o._native.OMX_E_INVALID


def test_param_blob_layout():
    b = param_blob([7, "n1", 2.5, None, True], {"x": 3})
    raw = b.tobytes()
    n = int(np.frombuffer(raw[:4], np.uint32)[0])
    assert n == 6 and len(raw) % 8 == 0


@pytest.mark.gpu
def test_packed_execute_on_device(match_test_db_json):
    """omx_execute_packed with a parameter buffer against omx_execute with omx_value parameters."""
    import orientdb_amd as o
    from orientdb_amd.graph import records_arrays
    L = o._native.lib()
    g = o.GraphSnapshot.from_blob(graph_blob(*records_arrays(match_test_db_json), device=0))
    q = "match {class:Person, as:person, where:(name = ? or name = :other)} return person"
    want = o.OMatchStatement(q).execute(g, "n1", other="n2")
    st = o.OMatchStatement(q)
    pb = param_blob(["n1"], {"other": "n2"})
    r = C.c_void_p()
    o._native.check(L.omx_execute_packed(g.handle, st._h, 0, 0, -1, 0, 1, None, pb.ctypes.data_as(C.c_void_p),
                                         pb.nbytes, C.byref(r)))
    try:
        got = o.OMatchStatement._collect(r, True)
    finally:
        L.omx_result_free(r)
    assert len(got) == len(want) == 2
    assert {d["person"] for d in got} == {d["person"] for d in want}
