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


def test_blob_version1_header_accepted(match_test_db_json):
    """Buffers of the 88-byte version-1 header (no edge records) still describe the same snapshot."""
    import orientdb_amd as o
    from orientdb_amd.graph import records_arrays
    arrays = records_arrays(match_test_db_json)
    g = o.GraphSnapshot.from_blob(graph_blob(*arrays, device=-1, version=1))
    ref = o.GraphSnapshot(*arrays, device=-1)
    for cls in ("V", "E", "Person", "TriangleE"):
        assert g.class_count(cls) == ref.class_count(cls)


EDGE_Q = "MATCH {class: TriangleV, as: a}.outE('TriangleE'){as: e}.inV(){as: b, where: (uid < 3)} RETURN a, e, b"


@pytest.fixture(scope="module")
def blob_edge_arrays():
    from orientdb_amd.graph import records_arrays
    from tests.test_gpu_edges import edge_db
    db = edge_db(n=60, n_knows=200, n_likes=50)
    a = records_arrays(db, edge_records=True)
    # one set given with its in CSR (+ in_edge_index), as a Java builder reading in_ ridbags would
    es = a[4][0]
    rp, col = np.asarray(es["out_rp"], np.int64), np.asarray(es["out_col"], np.int64)
    src = np.repeat(np.arange(len(rp) - 1), np.diff(rp))
    order = np.argsort(col, kind="stable")
    irp = np.zeros(len(rp), np.uint64)
    np.add.at(irp, col + 1, 1)
    es["in_rp"], es["in_col"], es["in_edge_index"] = np.cumsum(irp).astype(np.uint64), src[order], order
    return a


def test_blob_edge_records_equal_pointer_snapshot(blob_edge_arrays):
    import orientdb_amd as o
    a = blob_edge_arrays
    ref = o.GraphSnapshot(*a[:7], device=-1, edge_properties=a[7])
    g = o.GraphSnapshot.from_blob(graph_blob(*a[:7], device=-1, edge_properties=a[7]))
    for cls in ("V", "E", "Person", "Knows", "Likes"):
        assert g.class_count(cls) == ref.class_count(cls)
    assert ref.class_count("Knows") == 200 and ref.class_count("E") == 250
    for q in ("MATCH {class: Person, as: a}.outE('Knows'){as: e, where: (since > 2012)}.inV(){as: b} RETURN e",
              "MATCH {class: Knows, as: e, where: (since = 2015)}.outV(){as: a} RETURN e, a"):
        st = o.OMatchStatement(q)
        assert st.explain(g) == st.explain(ref)
        assert st.explain(g)["supported"]


def test_blob_edge_properties_need_records(blob_edge_arrays):
    import orientdb_amd as o
    a = blob_edge_arrays
    sets = [{k: v for k, v in es.items() if k not in ("edge_rids", "in_edge_index")} for es in a[4]]
    buf = graph_blob(*a[:4], sets, *a[5:7], device=-1, edge_properties=a[7])
    assert _create(buf) == o._native.OMX_E_INVALID


@pytest.mark.gpu
def test_blob_edge_records_on_device(blob_edge_arrays):
    """An edge-node MATCH on the blob snapshot (one set with a given in CSR) against the oracle."""
    import orientdb_amd as o
    from oracle.match_ref import MatchOracle, RefDB
    from tests.test_gpu_edges import edge_db
    from tests.test_gpu_parity import gpu_set, oracle_set
    a = blob_edge_arrays
    g = o.GraphSnapshot.from_blob(graph_blob(*a[:7], device=0, edge_properties=a[7]))
    ref = RefDB.from_json(edge_db(n=60, n_knows=200, n_likes=50))
    for q in ("MATCH {class: Person, as: b, where: (uid < 30)}.inE('Knows'){as: e, where: (since > 2010)}.outV(){as: a} RETURN a, e, b",
              "MATCH {class: Person, as: a}.outE('Knows'){as: e, where: (w < 0.5)}.inV(){as: b} RETURN $pathElements"):
        rs = o.OMatchStatement(q).execute(g)
        want = MatchOracle(ref, q).execute()
        cols = rs.columns if rs.columns[0] != "$pathElements" else None
        assert len(want) > 0 and gpu_set(rs) == oracle_set(want, cols)
