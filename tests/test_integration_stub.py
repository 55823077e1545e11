"""The INTEGRATION.md ctypes stub on CPU: it loads against the built library, and its
``_ip`` follows ``__ip_to_int`` (reference ``toeplitz.py:110-111``): IndexError below four
octets, extra octets ignored, values taken mod 2**32 by the byte masks (``:127-137``)."""
import numpy as np
import pytest

from integration_stub import load_stub


def test_stub_loads_and_binds():
    stub = load_stub()
    for name in ("rss_key_prepare", "rss_ctx_create", "rss_ctx_destroy", "rss_hash_host",
                 "rss_last_error"):
        assert hasattr(stub.LIB, name)
    key = stub._Key()
    assert stub.LIB.rss_key_prepare(bytes(range(40)), 40, key) == 0
    assert key.len == 40


def test_stub_ip_semantics():
    stub = load_stub()
    got = stub._ip(["1.2.3.4", "255.255.255.255", "1.2.3.4.5", "256.0.0.1", "0.0.0.-1"])
    want = [0x01020304, 0xFFFFFFFF, 0x01020304, (256 << 24 | 1) & 0xFFFFFFFF,
            (-1) & 0xFFFFFFFF]
    np.testing.assert_array_equal(got, np.array(want, dtype=np.uint32))
    with pytest.raises(IndexError):
        stub._ip(["1.2.3"])
