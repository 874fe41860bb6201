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
