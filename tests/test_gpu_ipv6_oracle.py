"""IPv6 element-wise against the C oracle at scale: every hash, queue
and count of millions of 36-byte tuples equals ``oracle_run_words`` -- the reference's
literal rotating-key loop (``toeplitz.py:46-69``) over the 36 input bytes, pinned on CPU to
``oracle_hash_bytes`` and the Microsoft IPv6 KAT (``tests/test_oracle.py``) -- with
``hash % htable % nqueues`` and the histogram of ``simulator.py:94-113``.  Covers the device
API (u32 / u16 / u8 queue columns, counts only, single-pass counts with the balanced tail,
many queues, misaligned input, accumulation), the host pipeline and the reference-compatible
``Toeplitz.compute_queues6``.  Before round 6 the IPv6 hashes were pinned by the KAT and by
sampled per-tuple checks only."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def native():
    from rss_simulator_nvidia_amd import _native
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need a gfx950 device")
    return _native


def _words(seed, n):
    rng = np.random.default_rng(seed)
    return rng.integers(0, 2**32, size=(n, 9), dtype=np.uint64).astype(np.uint32)


@pytest.mark.parametrize("H,Q,width", [(128, 24, 8), (128, 24, 32), (512, 100, 16),
                                       (1 << 20, 1000, 16), (100, 7, 32), (1 << 30, 50000, 32),
                                       (64, 64, 8)])
def test_device_elementwise(native, oracle_lib, example_key, H, Q, width):
    n = (1 << 22) + 3
    host = _words(1000 + Q, n)
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream(dev).cuda_stream
    t = torch.from_numpy(host.view(np.int32).reshape(-1)).to(dev)
    h = torch.empty(n, dtype=torch.int32, device=dev)
    qt = {8: torch.uint8, 16: torch.int16, 32: torch.int32}[width]
    q = torch.empty(n, dtype=qt, device=dev)
    qn = native.queue_modulus(H, Q)[1]
    c = torch.full((qn,), 7, dtype=torch.int64, device=dev)
    flags = {8: native.FLAG_QUEUE_U8, 16: native.FLAG_QUEUE_U16, 32: 0}[width]
    native.hash6_device(native.prepare_key6(example_key), t.data_ptr(), n, H, Q, h.data_ptr(),
                        q.data_ptr(), c.data_ptr(), flags, s)
    torch.cuda.synchronize()
    ho, qo, co = oracle_lib.run_words(example_key, host, H, Q)
    np.testing.assert_array_equal(h.cpu().numpy().view(np.uint32), ho)
    qv = q.cpu().numpy()
    if width != 8:
        qv = qv.view(np.uint16 if width == 16 else np.uint32)
    qv = qv.astype(np.uint32)
    np.testing.assert_array_equal(qv, qo)
    np.testing.assert_array_equal(c.cpu().numpy().view(np.uint64), co[:qn])


def test_single_pass_counts_only_and_accumulate(native, oracle_lib, example_key):
    """rss_hash6_device_ws (single-pass counts, balanced tail past 2^24 tuples) over stale
    counts, then a counts-only launch accumulating onto them, on a 4-byte-misaligned copy."""
    n, H, Q = (1 << 24) + 5, 128, 24
    host = _words(77, n)
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream(dev).cuda_stream
    flat = torch.from_numpy(host.view(np.int32).reshape(-1)).to(dev)
    key6 = native.prepare_key6(example_key)
    ho, qo, co = oracle_lib.run_words(example_key, host, H, Q)
    ws = torch.zeros(native.counts_workspace_bytes(H, Q) // 8, dtype=torch.int64, device=dev)
    h = torch.empty(n, dtype=torch.int32, device=dev)
    q = torch.empty(n, dtype=torch.uint8, device=dev)
    c = torch.full((Q,), 99, dtype=torch.int64, device=dev)
    native.hash6_device(key6, flat.data_ptr(), n, H, Q, h.data_ptr(), q.data_ptr(), c.data_ptr(),
                        native.FLAG_QUEUE_U8, s, ws.data_ptr())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(h.cpu().numpy().view(np.uint32), ho)
    np.testing.assert_array_equal(q.cpu().numpy().astype(np.uint32), qo)
    np.testing.assert_array_equal(c.cpu().numpy().view(np.uint64), co)
    assert int(ws.abs().sum()) == 0
    mis = torch.zeros(flat.numel() + 1, dtype=torch.int32, device=dev)
    mis[1:] = flat
    native.hash6_device(key6, mis.data_ptr() + 4, n, H, Q, None, None, c.data_ptr(),
                        native.FLAG_ACCUMULATE, s)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(c.cpu().numpy().view(np.uint64), 2 * co)


def test_host_path_and_reference_api(native, oracle_lib, example_key):
    """The host pipeline (rss_hash6_host) and Toeplitz.compute_queues6, one and two
    contexts, against the oracle element by element."""
    from rss_simulator_nvidia_amd.toeplitz import Toeplitz
    n, H, Q = 1_000_003, 512, 24
    host = _words(5, n)
    ho, qo, co = oracle_lib.run_words(example_key, host, H, Q)
    ctx = native.HostContext(0)
    h, q, c = ctx.hash6(native.prepare_key6(example_key), host, H, Q)
    for got, want in ((h, ho), (q, qo), (c, co)):
        np.testing.assert_array_equal(got, want)
    ctx.close()
    tz = Toeplitz(example_key)
    for devices in (None, [0, 0]):
        h, q, c = tz.compute_queues6(host, H, Q, devices=devices)
        for got, want in ((h, ho), (q, qo), (c, co)):
            np.testing.assert_array_equal(got, want)


IPV6_CHUNK = 21 * 65536  # rss_hash6_host's slot: 48 MB of 36-byte tuples, rounded down to 64K


@pytest.mark.parametrize("pin_in,pin_out", [(False, False), (True, True), (True, False),
                                            (False, True)])
def test_host_pipeline_chunks_and_pinned_buffers(native, oracle_lib, example_key, pin_in,
                                                 pin_out):
    """rss_hash6_host runs the IPv4 host path's pipeline: three 1.38M-tuple chunks with a
    ragged tail through two staging slots and two streams, or straight from / into
    page-locked caller buffers, every element equal to the oracle's; then an indirection
    table on the same context."""
    n, H, Q = 2 * IPV6_CHUNK + 12345, 128, 24
    host = _words(31, n)
    ho, qo, co = oracle_lib.run_words(example_key, host, H, Q)
    src = host
    if pin_in:
        src = native.pinned_empty(host.shape, np.uint32)
        src[:] = host
    alloc = native.pinned_empty if pin_out else (lambda k, t: np.empty(k, t))
    out = (alloc(n, np.uint32), alloc(n, np.uint32))
    out[0].fill(0xDEADBEEF)
    ctx = native.HostContext(0)
    key6 = native.prepare_key6(example_key)
    h, q, c = ctx.hash6(key6, src, H, Q, out=out)
    assert h is out[0] and q is out[1]
    for got, want in ((h, ho), (q, qo), (c, co)):
        np.testing.assert_array_equal(got, want)
    table = (np.arange(H, dtype=np.uint32) * 7) % 5
    _, q2, c2 = ctx.hash6(key6, src, H, 5, want_hash=False, reta=table)
    np.testing.assert_array_equal(q2, table[ho % H])
    np.testing.assert_array_equal(c2, np.bincount(table[ho % H], minlength=5).astype(np.uint64))
    ctx.close()


@pytest.mark.parametrize("n", [0, 1, 2, 255, 16383, 16384, 16385, 70001])
def test_host_small_batches_and_switch(native, oracle_lib, example_key, n):
    """Batches around the small-batch switch (16384 tuples: the kernel reads the mapped
    staging in place) and one past it, IPv4 and IPv6 calls alternating on one context so
    each grows and reuses the other's staging."""
    ctx = native.HostContext(0)
    key6, key4 = native.prepare_key6(example_key), native.prepare_key(example_key)
    w6 = _words(n + 1, n)
    w4 = oracle_lib.generate(n + 2, 0, n)
    for _ in range(2):
        h, q, c = ctx.hash6(key6, w6, 100, 7)
        ho, qo, co = oracle_lib.run_words(example_key, w6, 100, 7)
        for got, want in ((h, ho), (q, qo), (c, co)):
            np.testing.assert_array_equal(got, want)
        h, q, c = ctx.hash(key4, w4, 100, 7)
        ho, qo, co = oracle_lib.run(example_key, w4, 100, 7)
        for got, want in ((h, ho), (q, qo), (c, co)):
            np.testing.assert_array_equal(got, want)
    ctx.close()


def test_compute_queues6_one_tuple_per_call(native, oracle_lib, example_key):
    """The reference-style per-row use of compute_queues6: single tuples on the small path,
    one call each, against the oracle (per-call time: tools/host6_probe.py)."""
    from rss_simulator_nvidia_amd.toeplitz import Toeplitz
    tz = Toeplitz(example_key)
    w = _words(9, 300)
    ho, qo, _ = oracle_lib.run_words(example_key, w, 128, 24)
    for i in range(len(w)):
        h, q, c = tz.compute_queues6(w[i:i + 1], 128, 24)
        assert int(h[0]) == int(ho[i]) and int(q[0]) == int(qo[i]) and int(c.sum()) == 1
