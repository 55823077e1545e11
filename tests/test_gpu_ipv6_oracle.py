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
