"""Embedded ridbag streams (oracle/ridbag_ref.py): encode/decode round trips and the header variants
the device decoder (orientdb_amd/csrc/ridbag.hip) must accept or refuse. CPU only."""
import random

import pytest

from oracle import ridbag_ref as R


@pytest.mark.parametrize("seed", range(10))
def test_round_trip(seed):
    rnd = random.Random(seed)
    rids = [(rnd.randrange(0, 40), rnd.randrange(0, 1 << 40)) for _ in range(rnd.randrange(0, 50))]
    uuid = bytes(rnd.randrange(256) for _ in range(16)) if seed % 2 else None
    s = R.encode_embedded(rids, uuid)
    assert len(s) == 1 + (16 if uuid else 0) + 4 + 10 * len(rids)  # ORidBag + OEmbeddedRidBag sizes
    assert R.decode(s) == rids


def test_layout_is_big_endian():
    s = R.encode_embedded([(11, 258)])
    assert s == bytes([1, 0, 0, 0, 1, 0, 11, 0, 0, 0, 0, 0, 0, 1, 2])


def test_refused_streams():
    with pytest.raises(ValueError):
        R.decode(R.encode_sbtree_pointer())
    with pytest.raises(ValueError):
        R.decode(R.encode_embedded([(1, 2), (3, 4)])[:-1])
    assert R.decode(b"") == []


def test_decoder_symbol_exported():
    import orientdb_amd._native as N
    assert N.lib().omx_ridbag_decode_csr is not None
