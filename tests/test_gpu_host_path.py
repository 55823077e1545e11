"""rss_hash_host on page-locked buffers: the direct-DMA pipeline (no staging copies)
must give exactly what the staged pipeline and the oracle give, for every mix of
pinned / pageable input and outputs, over several chunks with a ragged tail; and a call whose launch fails part-way
leaves nothing in flight."""
import time

import numpy as np
import pytest
from hooks import hooks

from rss_simulator_nvidia_amd.exceptions import DeviceError

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def native():
    from rss_simulator_nvidia_amd import _native
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need a gfx950 device")
    return _native


@pytest.fixture(scope="module")
def ctx(native):
    return native.HostContext(0)


N = (9 << 20) + 5  # four chunks of the pipeline, the last one ragged
# the pipeline's chunk for N (rss_host.hip, hash_host_pipeline): a quarter of the batch in
# 64K-tuple steps, between 256K tuples and the 48 MB slot (4M IPv4 tuples)
CHUNK = min(4 << 20, max(1 << 18, (-(-N // 4) + 65535) // 65536 * 65536))


@pytest.fixture(scope="module")
def expected(oracle_lib, example_key):
    tup = oracle_lib.generate(0x5EED, 3, N)
    h, q, c = oracle_lib.run(example_key, tup, 128, 24, threads=16)
    return tup, h, q, c


@pytest.mark.parametrize("pin_in,pin_out", [(True, True), (True, False), (False, True)])
def test_pinned_buffers_match_oracle(native, ctx, example_key, expected, pin_in, pin_out):
    tup, ho, qo, co = expected
    if pin_in:
        src = native.pinned_empty(tup.shape, np.uint32)
        src[:] = tup
    else:
        src = tup
    if pin_out:
        out = (native.pinned_empty(N, np.uint32), native.pinned_empty(N, np.uint32))
    else:
        out = (np.empty(N, np.uint32), np.empty(N, np.uint32))
    out[0].fill(0xDEADBEEF)
    key = native.prepare_key(example_key)
    h, q, c = ctx.hash(key, src, 128, 24, out=out)
    assert h is out[0] and q is out[1]
    np.testing.assert_array_equal(h, ho)
    np.testing.assert_array_equal(q, qo)
    np.testing.assert_array_equal(c, co)
    # the same buffers again: reuse across batches (the point of pinning once)
    h.fill(0)
    h, q, c = ctx.hash(key, src, 128, 24, out=out)
    np.testing.assert_array_equal(h, ho)
    assert int(c.sum()) == N


def test_pinned_slices_and_hash_only(native, ctx, example_key, expected):
    """Interior slices of one pinned allocation are still DMA'd directly; NULL queue
    output (hash only) and an odd offset into the pinned tuples."""
    tup, ho, _, _ = expected
    src = native.pinned_empty(tup.shape, np.uint32)
    src[:] = tup
    hbuf = native.pinned_empty(N + 7, np.uint32)
    key = native.prepare_key(example_key)
    h, q, c = ctx.hash(key, src[1:], 1, 1, want_queue=False, want_counts=False,
                       out=(hbuf[7:N + 6], None))
    assert q is None and c is None
    np.testing.assert_array_equal(h, ho[1:])


def test_pinned_empty_shapes(native):
    a = native.pinned_empty((3, 4), np.uint64)
    assert a.shape == (3, 4) and a.dtype == np.uint64 and a.flags.c_contiguous
    a[:] = 7
    assert int(a.sum()) == 84
    z = native.pinned_empty(0, np.uint32)
    assert z.shape == (0,)


@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0]])
def test_multi_context_host_batch_matches_oracle(native, example_key, expected, devices):
    """rss_hash_host_multi: contiguous ranges over several contexts (here all on cuda:0,
    each with its own streams and host thread) give exactly the single-device result."""
    tup, ho, qo, co = expected
    multi = native.MultiHostContext(devices)
    key = native.prepare_key(example_key)
    h, q, c = multi.hash(key, tup, 128, 24)
    np.testing.assert_array_equal(h, ho)
    np.testing.assert_array_equal(q, qo)
    np.testing.assert_array_equal(c, co)
    # page-locked outputs (direct DMA per range) and hash-only
    out = (native.pinned_empty(N, np.uint32), None)
    h2, q2, c2 = multi.hash(key, tup, 128, 24, want_queue=False, want_counts=False, out=out)
    assert q2 is None and c2 is None
    np.testing.assert_array_equal(h2, ho)
    multi.close()


@pytest.mark.parametrize("n", [0, 1, 2, 5, 4099])
def test_multi_context_small_and_ragged(native, oracle_lib, example_key, n):
    """Fewer tuples than contexts (empty ranges), ragged splits and an indirection table."""
    tup = oracle_lib.generate(99, 0, n)
    multi = native.MultiHostContext([0, 0, 0])
    key = native.prepare_key(example_key)
    h, q, c = multi.hash(key, tup, 100, 7)
    eh, eq, ec = oracle_lib.run(example_key, tup, 100, 7)
    np.testing.assert_array_equal(h, eh)
    np.testing.assert_array_equal(q, eq)
    np.testing.assert_array_equal(c, ec)
    reta = np.arange(64, dtype=np.uint32)[::-1] % 5
    h, q, c = multi.hash(key, tup, 64, 5, reta=reta)
    eh = oracle_lib.run(example_key, tup, 64, 5)[0]
    np.testing.assert_array_equal(q, reta[eh % 64])
    np.testing.assert_array_equal(c, np.bincount(reta[eh % 64], minlength=5).astype(np.uint64))
    multi.close()


@pytest.mark.parametrize("fail_at", [1, 2, 3])
@pytest.mark.parametrize("pinned", [True, False])
def test_failed_chunk_leaves_nothing_in_flight(native, example_key, expected, fail_at, pinned):
    """A launch that fails part-way through a host call (hooks fail_launch: the first, second
    or third chunk) reports the error, and the call has waited out the earlier
    chunks' copies before returning: the caller's page-locked outputs stop changing the
    moment it returns, and the next call on the same context gives the oracle's results."""
    tup, ho, qo, co = expected
    key = native.prepare_key(example_key)
    if pinned:
        src = native.pinned_empty(tup.shape, np.uint32)
        src[:] = tup
        out = (native.pinned_empty(N, np.uint32), native.pinned_empty(N, np.uint32))
    else:
        src, out = tup, (np.empty(N, np.uint32), np.empty(N, np.uint32))
    with hooks(fail_launch=fail_at):
        hctx = native.HostContext(0)
        out[0].fill(0xDEADBEEF)
        with pytest.raises(DeviceError, match="fail_launch"):
            hctx.hash(key, src, 128, 24, out=out)
        snap = out[0].copy()
        time.sleep(0.05)
        np.testing.assert_array_equal(out[0], snap)
        if pinned:  # chunks before the failed one were written directly, none after
            done = CHUNK * (fail_at - 1)
            np.testing.assert_array_equal(out[0][:done], ho[:done])
            assert (out[0][done:] == 0xDEADBEEF).all()
        h, q, c = hctx.hash(key, src, 128, 24, out=out)
        np.testing.assert_array_equal(h, ho)
        np.testing.assert_array_equal(q, qo)
        np.testing.assert_array_equal(c, co)
        hctx.close()


def test_failed_small_batch_then_recovers(native, example_key, expected):
    """The small-batch path (<= 16384 tuples) after a failed launch on the same context."""
    tup, ho, qo, _ = expected
    key = native.prepare_key(example_key)
    with hooks(fail_launch=1):
        hctx = native.HostContext(0)
        with pytest.raises(DeviceError, match="fail_launch"):
            hctx.hash(key, tup[:1000], 128, 24)
        h, q, c = hctx.hash(key, tup[:1000], 128, 24)
        np.testing.assert_array_equal(h, ho[:1000])
        np.testing.assert_array_equal(q, qo[:1000])
        assert int(c.sum()) == 1000
        hctx.close()
