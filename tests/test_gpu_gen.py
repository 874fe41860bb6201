"""The device RMAT generator (orientdb_amd/csrc/gen.hip) builds exactly the arrays of the host
generator (gen.cpp): full graphs and 1-D partitions (out and in rows), simple and multigraph. The host
generator is itself pinned by tests/test_generator.py and tests/test_partition_cpu.py."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("scale,simple,seed", [(8, True, 8), (8, False, 3), (14, True, 14), (16, False, 16)])
def test_device_rmat_equals_host(scale, simple, seed, monkeypatch):
    from orientdb_amd.graph import rmat_csr
    rp_d, col_d = rmat_csr(scale, 16, seed, simple, device=0)
    monkeypatch.setenv("OMX_GEN_HOST", "1")
    rp_h, col_h = rmat_csr(scale, 16, seed, simple, device=0)
    assert np.array_equal(rp_d, rp_h)
    assert np.array_equal(col_d, col_h)


@pytest.mark.parametrize("world", [3, 4])
@pytest.mark.parametrize("simple", [True, False])
def test_device_rmat_partitions_equal_host(world, simple, monkeypatch):
    from orientdb_amd.graph import partition_range, rmat_partition
    V = 1 << 12
    for r in range(world):
        lo, hi = partition_range(V, r, world)
        monkeypatch.delenv("OMX_GEN_HOST", raising=False)
        dev = rmat_partition(12, lo, hi, 16, 5, simple, device=0)
        monkeypatch.setenv("OMX_GEN_HOST", "1")
        host = rmat_partition(12, lo, hi, 16, 5, simple, device=0)
        for a, b in zip(dev, host):
            assert np.array_equal(a, b)


def test_device_rmat_empty_partition():
    from orientdb_amd.graph import rmat_partition
    orp, ocol, irp, icol = rmat_partition(6, 64, 64, device=0)
    assert orp.tolist() == [0] and irp.tolist() == [0] and len(ocol) == 0 and len(icol) == 0
