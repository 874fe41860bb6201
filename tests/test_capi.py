"""The C-ABI library loads and exports every symbol include/omx/match.h declares (no device calls)."""
import ctypes
import os
import re

from tests.conftest import ROOT


def header_symbols():
    with open(os.path.join(ROOT, "include", "omx", "match.h")) as f:
        text = f.read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(omx_[a-z_0-9]+)\s*\(", text)))


def test_library_exports_every_header_symbol():
    from orientdb_amd import _native
    lib = ctypes.CDLL(_native.LIB_PATH)
    syms = header_symbols()
    assert len(syms) >= 20
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing


def test_bindings_cover_header():
    from orientdb_amd import _native
    assert set(header_symbols()) == set(_native.SIGNATURES)


def test_errors_are_reported():
    import orientdb_amd as o
    import pytest
    with pytest.raises(o.OmxParseError):
        o.OMatchStatement("match {class:Person, as: p return p")
    with pytest.raises(o.OmxParseError):
        o.OMatchStatement("update V set x = 1")
    with pytest.raises(o.OmxUnsupported):  # valid SQL the legacy executor keeps (only SELECT expand() is taken)
        o.OMatchStatement("select from V")


def test_optional_validation_is_a_parse_error(match_test_db_json):
    """Pattern.validate (P/Pattern.java:48-65): optional nodes only as right terminals."""
    import orientdb_amd as o
    import pytest
    g = o.GraphSnapshot.from_records(match_test_db_json, device=-1)
    st = o.OMatchStatement("match {class:Person, as:a, optional:true}-Friend->{as:b} return a")
    with pytest.raises(o.OmxParseError):
        st.explain(g)


def test_host_comm_created_without_a_device():
    """omx_comm_create_host checks its callbacks and ranks (no device, no collective at creation)."""
    import ctypes as C

    import orientdb_amd as o
    from orientdb_amd import dist
    L = o._native.lib()
    h = C.c_void_p()
    hc = dist._HostCollectives(None, dist._ALLG(lambda *a: 0), dist._A2AV(lambda *a: 0), dist._ABRT(lambda c: None))
    assert L.omx_comm_create_host(1, 2, C.byref(hc), C.byref(h)) == 0
    assert L.omx_comm_rank(h) == 1 and L.omx_comm_world(h) == 2
    L.omx_comm_destroy(h)
    assert L.omx_comm_create_host(2, 2, C.byref(hc), C.byref(h)) == o._native.OMX_E_INVALID
    bad = dist._HostCollectives(None, dist._ALLG(), dist._A2AV(lambda *a: 0), dist._ABRT())
    assert L.omx_comm_create_host(0, 2, C.byref(bad), C.byref(h)) == o._native.OMX_E_INVALID
